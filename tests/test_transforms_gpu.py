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


def run(buf, off, lens, fmt, t: Transforms, block_fmt=None, flags=0):
    d = decode(BlockBatch.from_host(buf, off, lens, "cuda", fmt, flags, block_format=block_fmt))
    g = apply_transforms(d, t).to_host()
    o = oracle.transform_batch(oracle.decode_batch(buf, off, lens, fmt, block_fmt, flags), t.synthetic_seq_num,
                               t.hide_obsolete_points, t.synthetic_prefix, t.synthetic_suffix, t.split,
                               src=(buf, off, lens, fmt, block_fmt, flags))
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


@pytest.mark.parametrize("seed", range(6))
def test_row_prefix_semantics_short_keys_and_split(seed):
    """Row blocks under the transforms rowblk.Iter applies with the prefix
    inside fullKey (rowblk_iter.go:259-263,400,1168-1199): raw keys shorter than
    8 B made valid by the prefix, Split over prefix ++ key (testkeys '@' in the
    prefix only, cockroachkvs version-length bytes reaching into the prefix),
    hidden points and value prefixes of kinds taken from the prefix."""
    from test_oracle_row_transforms import PREFIXES, raw_block, random_raw_keys, random_values
    rng = random.Random(500 + seed)
    flags = [0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_VALUE_PREFIX | N.PBL_ROW_NO_VALUER][seed % 3]
    blocks = []
    for _ in range(120):
        n = rng.randint(1, 80)
        blocks.append(raw_block(random_raw_keys(rng, n), random_values(rng, n), rng.choice([1, 2, 3, 16])))
    buf, off, lens = pack(blocks)
    for prefix in PREFIXES:
        for suffix, split in ((b"", 0), (b"@9", N.PBL_SPLIT_TESTKEYS), (b"\x00" * 7 + b"\x07\x09", N.PBL_SPLIT_CRDB)):
            t = Transforms(rng.choice([0, 77]), rng.random() < 0.5, prefix, suffix, split)
            g, o = run(buf, off, lens, N.PBL_FMT_ROW, t, flags=flags)
            assert_same(g, o, f"seed={seed} prefix={prefix!r} suffix={suffix!r}")


def test_row_short_key_made_valid_on_gpu():
    from test_oracle_row_transforms import raw_block
    keys = [b"k" * 8 + (5 << 8 | 1).to_bytes(8, "little"), b"\x07\x08\x09", b"\x07\x08\x09\x0a"]
    blk = raw_block(keys, [b"\x00v0", b"\x00v1", b""], 2)
    buf, off, lens = pack([blk, blk])
    prefix = b"PQR\x01\x01\x00\x00\x00"  # kinds of the short keys: prefix[3] and prefix[4] (SET)
    g, o = run(buf, off, lens, N.PBL_FMT_ROW, Transforms(synthetic_prefix=prefix), flags=N.PBL_ROW_VALUE_PREFIX)
    assert_same(g, o, "short key made valid")
    # the third key becomes SET with an empty value: Go's i.val[0] panics -> corrupt block
    assert g["n_bad_blocks"] == 2 and g["status_mask"] == 1 << N.PBL_CORRUPT_BOUNDS
    g, o = run(buf, off, lens, N.PBL_FMT_ROW, Transforms(synthetic_prefix=b"PQR\x02\x02\x00\x00\x00"),
               flags=N.PBL_ROW_VALUE_PREFIX)
    assert_same(g, o, "short key made valid (kind MERGE)")
    assert g["blk_status"].tolist() == [0, 0] and g["key_bytes"][:3].tobytes() == b"PQR"
    assert g["n_kv"] == 6 and not (g["kv_flags"] & N.PBL_KV_INVALID_KEY).any()
