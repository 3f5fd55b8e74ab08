"""Device transforms (pbl_transform_batch, pebble_amd/transforms.py) against
the oracle's restatement (oracle.transform_batch, pinned by the reference's
transform scans in tests/test_oracle_transforms.py): bit-exact on every output
array, over the reference's transform blocks, random row and colblk batches
(both key schemas, obsolete points, invalid keys, corrupt blocks) and a
config-3-shaped batch; plus the capacity-overflow contract."""
import json
import os
import random

import numpy as np
import pytest

import oracle
from colutil import build_block, random_rows
from pebble_amd import _native as N
from pebble_amd.batch import BlockBatch, Capacity, decode
from pebble_amd.colblk import SCHEMA_CRDB1, SCHEMA_DEFAULT, gen_col_blocks
from pebble_amd.rowblk import gen_row_blocks
from pebble_amd.transforms import Transforms, apply_transforms
from test_oracle_transforms import TRANSFORMS, check_scan, encode_rows, forward
from test_rowblk_gpu import ARRAYS, assert_same, pack, random_block

pytestmark = pytest.mark.gpu


def run(buf, off, lens, fmt, t: Transforms, block_fmt=None):
    d = decode(BlockBatch.from_host(buf, off, lens, "cuda", fmt, 0, block_format=block_fmt))
    g = apply_transforms(d, t).to_host()
    o = oracle.transform_batch(oracle.decode_batch(buf, off, lens, fmt, block_fmt), t.synthetic_seq_num,
                               t.hide_obsolete_points, t.synthetic_prefix, t.synthetic_suffix, t.split)
    return g, o


def test_reference_transform_scans_on_gpu():
    for tc in TRANSFORMS:
        blk = encode_rows(tc["rows"])
        buf, off, lens = pack([blk])
        for it in tc["iters"]:
            t = Transforms(it["seq_num"], it["hide_obsolete"], bytes.fromhex(it["prefix"]), bytes.fromhex(it["suffix"]),
                           N.PBL_SPLIT_TESTKEYS)
            g, o = run(buf, off, lens, SCHEMA_DEFAULT, t)
            assert_same(g, o, f"{tc['source']} iter@{it['line']}")
            check_scan(forward(g), it["forward"], f"{tc['source']} iter@{it['line']}")


TRANSFORM_SETS = [
    Transforms(),
    Transforms(synthetic_seq_num=1234),
    Transforms(hide_obsolete_points=True),
    Transforms(synthetic_prefix=b"foo_"),
    Transforms(synthetic_seq_num=(1 << 56) - 1, hide_obsolete_points=True, synthetic_prefix=b"\x00pre\xff"),
]


@pytest.mark.parametrize("ti", range(len(TRANSFORM_SETS)))
def test_random_row_batches(ti):
    rng = random.Random(40 + ti)
    blocks = []
    for _ in range(250):
        b = bytearray(random_block(rng)[0])
        if rng.random() < 0.1 and len(b) > 4:
            b[rng.randrange(len(b))] ^= 0x55  # some corrupt blocks
        blocks.append(bytes(b))
    g, o = run(*pack(blocks), N.PBL_FMT_ROW, TRANSFORM_SETS[ti])
    assert_same(g, o, f"row transforms {ti}")


@pytest.mark.parametrize("schema,split", [(SCHEMA_DEFAULT, N.PBL_SPLIT_TESTKEYS), (SCHEMA_CRDB1, N.PBL_SPLIT_CRDB)])
@pytest.mark.parametrize("ti", range(4))
def test_random_colblk_batches(schema, split, ti):
    rng = random.Random(schema * 10 + ti)
    blocks = []
    for _ in range(80):
        rows = random_rows(rng, schema, rng.choice([1, 5, 17, 100, 300]), shared=rng.choice([0, 3]),
                           val_len=(0, rng.choice([3, 50])))
        blocks.append(build_block(schema, rows, rng.choice([1, 4, 16]))[0])
    t = [Transforms(synthetic_suffix=b"@10" if schema == SCHEMA_DEFAULT else b"\x00\x00\x00\x00\x00\x00\x00\x05\x09",
                    split=split),
         Transforms(synthetic_seq_num=99, hide_obsolete_points=True, synthetic_prefix=b"p/",
                    synthetic_suffix=b"@7" if schema == SCHEMA_DEFAULT else b"\x01", split=split),
         Transforms(hide_obsolete_points=True),
         Transforms(synthetic_prefix=b"x" * 40, split=split)][ti]
    g, o = run(*pack(blocks), schema, t)
    assert_same(g, o, f"colblk schema={schema} transforms {ti}")


def test_mixed_config3_shape_and_overflow():
    buf, off, lens, n = gen_col_blocks(5, 2000)
    t = Transforms(synthetic_seq_num=7, synthetic_prefix=b"tenant/")
    g, o = run(buf, off, lens, SCHEMA_CRDB1, t)
    assert_same(g, o, "config-3 shape")
    assert g["n_kv"] == n and np.all((g["trailer"] >> np.uint64(8)) == 7)
    # too small an output: sizes only, every decodable block reports OVERFLOW
    d = decode(BlockBatch.from_host(buf, off, lens, "cuda", SCHEMA_CRDB1, 0))
    x = apply_transforms(d, t, cap=Capacity(kv=10, key=10, val=10, rst=10**9))
    tt = x.read_totals()
    assert tt.status_mask & (1 << N.PBL_OVERFLOW) and tt.n_kv == n


def test_row_config2_shape_seqnum_property():
    buf, off, lens, n = gen_row_blocks(9, 4096, 32768, 16, 16, 100)
    d = decode(BlockBatch.from_host(buf, off, lens, "cuda"))
    h = d.to_host()
    x = apply_transforms(d, Transforms(synthetic_seq_num=12345, synthetic_prefix=b"pp")).to_host()
    assert x["n_kv"] == n and x["key_bytes_total"] == h["key_bytes_total"] + 2 * n
    assert np.array_equal(x["trailer"] & np.uint64(0xFF), h["trailer"] & np.uint64(0xFF))
    assert np.all((x["trailer"] >> np.uint64(8)) == 12345)
    assert np.array_equal(x["val_bytes"], h["val_bytes"]) and np.array_equal(x["restarts"], h["restarts"])
