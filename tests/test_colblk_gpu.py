"""Parity of the HIP colblk decoder (through the C-ABI) against the CPU oracle and
the reference's own data blocks: bit-exact on every array of the output
contract (include/pebble_amd.h)."""
import json
import os
import random

import numpy as np
import pytest

import oracle
from colutil import build_block, random_rows
from pebble_amd import _native as N
from pebble_amd.colblk import SCHEMA_CRDB1, SCHEMA_DEFAULT, NewDataBlockIter, gen_col_blocks
from pebble_amd.rowblk import CorruptionError, Transforms, gen_row_blocks, kvs_of_block
from test_rowblk_gpu import ARRAYS, assert_same, pack

pytestmark = pytest.mark.gpu
# the colblk paths: the default two-pass wave form (colblk_wave.hip.h; fixed and
# variable-length stages), the pipeline and the one-block-per-workgroup kernel
KERNELS = {"wave": 0, "wave_varlen": N.PBL_BATCH_VARLEN, "pipe": N.PBL_KERNEL_PIPE, "single": N.PBL_KERNEL_SINGLE}
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "colblk_golden.json")


def gpu_decode(buf, off, lens, fmt, block_fmt=None, cap=None, flags=0):
    from pebble_amd.batch import BlockBatch, decode
    b = BlockBatch.from_host(buf, off, lens, "cuda", fmt, flags, block_format=block_fmt)
    return decode(b, cap=cap).to_host()


def check(buf, off, lens, fmt, block_fmt=None, ctx="", flags=0):
    o = oracle.decode_batch(buf, off, lens, fmt, block_fmt, flags)
    g = gpu_decode(buf, off, lens, fmt, block_fmt, flags=flags)
    assert_same(g, o, ctx)
    return g


def test_reference_blocks_on_gpu():
    with open(GOLDEN) as f:
        cases = json.load(f)["data_blocks"]
    for schema in (SCHEMA_DEFAULT, SCHEMA_CRDB1):
        cs = [c for c in cases if (c["schema"] == "crdb1") == (schema == SCHEMA_CRDB1)]
        blocks = [bytes.fromhex(c["block"]) for c in cs]
        g = check(*pack(blocks), schema, ctx=f"golden schema={schema}")
        for b, c in enumerate(cs):
            kvs = kvs_of_block(g, b)
            exp = [bytes.fromhex(r["key"]) for r in c["rows"]]
            assert [kv.user_key for kv in kvs] == exp, c["name"]
            assert [kv.trailer for kv in kvs] == [r["trailer"] for r in c["rows"]], c["name"]
            assert [kv.value for kv in kvs] == [bytes.fromhex(r["value"]) for r in c["rows"]], c["name"]


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("schema", [SCHEMA_DEFAULT, SCHEMA_CRDB1])
def test_random_blocks(schema, kernel):
    rng = random.Random(schema)
    blocks, exps = [], []
    for i in range(120):
        n = rng.choice([1, 2, 5, 16, 17, 100, 255, 256, 257, 300, 700])
        rows = random_rows(rng, schema, n, shared=rng.choice([0, 2, 7]), val_len=(0, rng.choice([1, 40, 300])))
        blk, exp = build_block(schema, rows, rng.choice([1, 2, 16, 64]))
        blocks.append(blk)
        exps.append(exp)
    for align in (16, 8, 1):
        g = check(*pack(blocks, align), schema, ctx=f"random schema={schema} align={align} {kernel}",
                  flags=KERNELS[kernel])
        for b in (0, 7, 63, 119):
            kvs = kvs_of_block(g, b)
            assert [(kv.user_key, kv.trailer, kv.value, kv.flags) for kv in kvs] == [e[:4] for e in exps[b]]


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_large_key_regions_and_chunks(kernel):
    """Key columns past the LDS stage (global-read path), > 256 rows per block
    (chunked key placement) and chunks whose keys exceed the LDS key buffer."""
    rng = random.Random(77)
    blocks = []
    for schema, n, kl, shared in [(SCHEMA_CRDB1, 40, (300, 600), 0), (SCHEMA_DEFAULT, 900, (1, 30), 5),
                                  (SCHEMA_DEFAULT, 300, (60, 90), 40), (SCHEMA_CRDB1, 2000, (4, 12), 2),
                                  (SCHEMA_DEFAULT, 30, (1000, 1500), 900)]:
        rows = random_rows(rng, schema, n, key_len=kl, shared=shared, val_len=(0, 8))
        blocks.append((schema, build_block(schema, rows, 16)[0]))
    for schema in (SCHEMA_DEFAULT, SCHEMA_CRDB1):
        bl = [b for s, b in blocks if s == schema]
        g = check(*pack(bl), schema, ctx=f"large schema={schema} {kernel}", flags=KERNELS[kernel])


def test_mixed_row_and_colblk_batch():
    """Config 4 shape: per-block formats in one batch (block_format[])."""
    rb, ro, rl, rn = gen_row_blocks(4, 16, 32768, 16, 16, 100)
    cb, co, cl, cn = gen_col_blocks(4, 16)
    blocks, fmts = [], []
    for i in range(16):
        blocks.append(bytes(rb[ro[i]:ro[i] + rl[i]]))
        fmts.append(N.PBL_FMT_ROW)
        blocks.append(bytes(cb[co[i]:co[i] + cl[i]]))
        fmts.append(N.PBL_FMT_COL_CRDB1)
    rng = random.Random(3)
    rows = random_rows(rng, SCHEMA_DEFAULT, 100)
    blocks.append(build_block(SCHEMA_DEFAULT, rows)[0])
    fmts.append(N.PBL_FMT_COL_DEFAULT)
    g = check(*pack(blocks), 0, np.array(fmts, np.uint8), ctx="mixed")
    assert g["n_kv"] == rn + cn + 100


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_corrupt_and_fuzzed_colblk(kernel):
    rng = random.Random(11)
    rows = random_rows(rng, SCHEMA_CRDB1, 80)
    base, _ = build_block(SCHEMA_CRDB1, rows)
    blocks = [base[:10], base[:len(base) // 2], base]
    for i in range(300):
        b = bytearray(base)
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(len(b))] = rng.randrange(256)
        blocks.append(bytes(b))
    g = check(*pack(blocks), SCHEMA_CRDB1, ctx=f"fuzz {kernel}", flags=KERNELS[kernel])
    assert g["n_bad_blocks"] > 0
    # the wrong schema for the block is a header corruption
    g = check(*pack([base]), SCHEMA_DEFAULT, ctx="wrong schema")
    assert g["blk_status"][0] == N.PBL_CORRUPT_COLBLK_HEADER


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_colblk_overflow_retry(kernel):
    from pebble_amd.batch import BlockBatch, Capacity, decode, size_batch
    buf, off, lens, n = gen_col_blocks(8, 32)
    o = oracle.decode_batch(buf, off, lens, SCHEMA_CRDB1)
    g = gpu_decode(buf, off, lens, SCHEMA_CRDB1, cap=Capacity(kv=10, key=10, val=10, rst=10), flags=KERNELS[kernel])
    assert_same(g, o, f"overflow retry {kernel}")
    b = BlockBatch.from_host(buf, off, lens, "cuda", SCHEMA_CRDB1, KERNELS[kernel])
    assert_same(decode(b, exact=True).to_host(), o, f"exact {kernel}")


def test_new_data_block_iter():
    with open(GOLDEN) as f:
        c = next(c for c in json.load(f)["data_blocks"] if c["name"].startswith("simple:41"))
    it = NewDataBlockIter(bytes.fromhex(c["block"]), SCHEMA_DEFAULT)
    kv = it.First()
    assert kv.user_key == b"a@10" and kv.value == b"apple"
    keys = [kv.user_key]
    while (kv := it.Next()) is not None:
        keys.append(kv.user_key)
    assert keys == [bytes.fromhex(r["key"]) for r in c["rows"]]
    assert it.SeekGE(b"c").user_key == b"c@9"  # testkeys order: newer suffixes first
    it2 = NewDataBlockIter(bytes.fromhex(c["block"]), SCHEMA_DEFAULT,
                           transforms=Transforms(hide_obsolete_points=True))
    ks = []
    kv = it2.First()
    while kv is not None:
        ks.append(kv.user_key)
        kv = it2.Next()
    assert b"d@11" not in ks  # the obsolete row is hidden
    with pytest.raises(CorruptionError):
        NewDataBlockIter(bytes.fromhex(c["block"])[:12], SCHEMA_DEFAULT)


def test_codec_columns_in_device_blocks():
    """The per-codec columns of the reference's codec tests (uints, raw_bytes,
    bitmap, prefix_bytes; tests/test_oracle_codecs.py) embedded in data blocks
    and decoded on the device: bit-exact with the oracle, and each embedded
    column yields the values the reference's test wrote."""
    from test_oracle_codecs import decoded_field, embedded_blocks, expected_field
    blocks = embedded_blocks()
    for align in (8, 16):
        g = check(*pack([b for _, _, b in blocks], align), SCHEMA_DEFAULT, ctx=f"codecs align={align}")
        for i, (codec, e, _) in enumerate(blocks):
            kvs = [(kv.user_key, kv.trailer, kv.value, kv.flags, 0) for kv in kvs_of_block(g, i)]
            assert decoded_field(codec, kvs) == expected_field(codec, e), e["source"]
