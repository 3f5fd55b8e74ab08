"""HideObsoletePoints fused into the decode (batch flag PBL_ROW_HIDE_OBSOLETE:
rowblk_iter.go:1168-1179) on the device against the oracle's decode under the
same flag (tests/test_oracle_hide.py pins that against the transform
restatement): bit-exact on every output array for random blocks, versioned
keys whose shared prefix reaches the kind byte, value prefixes, blocks past
the fast path's limits and past the 32 KiB stage; config-2 blocks (no obsolete
points) decode as without the flag.  Colblk batches (the isObsolete bitmap,
data_block.go:1680-1697) against oracle.transform_batch(hide) over the
oracle's plain decode."""
import random

import numpy as np
import pytest

import oracle
from pebble_amd import _native as N
from pebble_amd.batch import BlockBatch, decode
from pebble_amd.rowblk import gen_row_blocks
from colutil import build_block, random_rows
from pebble_amd.colblk import SCHEMA_CRDB1, SCHEMA_DEFAULT
from rowutil import mvcc_block
from test_rowblk_gpu import assert_same, pack, random_block

pytestmark = pytest.mark.gpu
HIDE = N.PBL_ROW_HIDE_OBSOLETE


def check(buf, off, lens, flags, ctx):
    o = oracle.decode_batch(buf, off, lens, 0, None, flags | HIDE)
    g = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, flags | HIDE)).to_host()
    assert_same(g, o, ctx)
    return g


@pytest.mark.parametrize("flags", [0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_VALUE_PREFIX | N.PBL_ROW_NO_VALUER])
def test_random_and_versioned_blocks(flags):
    rng = random.Random(60 + flags)
    blocks = [random_block(rng)[0] for _ in range(200)]
    blocks += [mvcc_block(rng, rng.randint(1, 380), rng.choice([1, 2, 16, 33]), rng.random() < 0.5,
                          rng.random() < 0.7) for _ in range(200)]
    rng.shuffle(blocks)
    g = check(*pack(blocks), flags, f"hide flags={flags}")
    plain = oracle.decode_batch(*pack(blocks), 0, None, flags)
    assert g["n_kv"] < plain["n_kv"]


def test_general_path_blocks():
    # more entries than a slot holds (288 / 336), runs longer than 16, corrupt blocks
    rng = random.Random(61)
    blocks = [mvcc_block(rng, 900, 1, False, True), mvcc_block(rng, 600, 64, True, True),
              mvcc_block(rng, 300, 40, False, False)]
    for _ in range(40):
        b = bytearray(mvcc_block(rng, rng.randint(1, 200), 16))
        b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        blocks.append(bytes(b))
    check(*pack(blocks), N.PBL_ROW_VALUE_PREFIX, "general")
    check(*pack(blocks), 0, "general, no prefix")


def test_blocks_past_the_stage():
    rng = random.Random(62)
    blocks = [mvcc_block(rng, 2500, 16) for _ in range(3)] + [mvcc_block(rng, 100, 16) for _ in range(20)]
    assert max(len(b) for b in blocks) > 32768
    check(*pack(blocks), 0, "big blocks")


def test_config2_without_obsolete_points_is_unchanged():
    buf, off, lens, n = gen_row_blocks(3, 3000, 32768, 16, 16, 100)
    a = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, HIDE)).to_host()
    b = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, 0)).to_host()
    for k in ("trailer", "kv_flags", "entry_off", "key_off", "val_off", "key_bytes", "val_bytes", "restarts",
              "blk_kv_base", "blk_key_base", "blk_val_base", "blk_status"):
        assert np.array_equal(a[k], b[k]), k
    assert a["n_kv"] == n


@pytest.mark.parametrize("schema", [SCHEMA_DEFAULT, SCHEMA_CRDB1])
def test_colblk_batches(schema):
    rng = random.Random(70 + schema)
    blocks = []
    for _ in range(120):
        rows = random_rows(rng, schema, rng.choice([1, 5, 17, 100, 300, 700]), shared=rng.choice([0, 3]),
                           val_len=(0, rng.choice([3, 50, 400])))
        blocks.append(build_block(schema, rows, rng.choice([1, 4, 16]))[0])
    for i in range(0, 120, 23):  # a few corrupt blocks stay failed
        b = bytearray(blocks[i])
        b[rng.randrange(len(b))] ^= 0x5A
        blocks[i] = bytes(b)
    buf, off, lens = pack(blocks)
    plain = oracle.decode_batch(buf, off, lens, schema, None, 0)
    o = oracle.transform_batch(plain, 0, True)
    for seq in (0, 4242):
        bb = BlockBatch.from_host(buf, off, lens, "cuda", schema, HIDE)
        bb.synthetic_seq_num = seq
        g = decode(bb).to_host()
        assert_same(g, oracle.transform_batch(plain, seq, True) if seq else o, f"colblk schema={schema} seq={seq}")
    assert 0 < g["n_kv"] < plain["n_kv"]


def test_colblk_config3_shaped():
    from pebble_amd.colblk import gen_col_blocks
    buf, off, lens, n = gen_col_blocks(1, 64, 32768)
    o = oracle.transform_batch(oracle.decode_batch(buf, off, lens, N.PBL_FMT_COL_CRDB1, None, 0), 0, True)
    g = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_CRDB1, HIDE)).to_host()
    assert_same(g, o, "config-3 shaped")


@pytest.mark.parametrize("flags", [0, N.PBL_ROW_VALUE_PREFIX])
def test_mixed_batches(flags):
    """Mixed row + colblk batches under the flag (config 4's shape): colblk rows
    by their isObsolete bit, row entries by their trailer's obsolete bit, every
    block placed by one look-back over the batch order; against the oracle's
    fused decode (pinned by test_oracle_hide.py), and the size pass agrees."""
    from pebble_amd.batch import size_batch
    rng = random.Random(71 + flags)
    blocks, fmts = [], []
    for i in range(300):
        k = rng.randrange(4)
        if k == 0:
            blocks.append(mvcc_block(rng, rng.randint(1, 300), rng.choice([1, 2, 16, 33]), rng.random() < 0.5,
                                     rng.random() < 0.7))
            fmts.append(N.PBL_FMT_ROW)
        elif k == 1:
            blocks.append(random_block(rng)[0])
            fmts.append(N.PBL_FMT_ROW)
        else:
            schema = SCHEMA_DEFAULT if k == 2 else SCHEMA_CRDB1
            rows = random_rows(rng, schema, rng.choice([1, 5, 17, 100, 300]), shared=rng.choice([0, 3]),
                               val_len=(0, rng.choice([3, 50, 400])))
            blocks.append(build_block(schema, rows, rng.choice([1, 4, 16]))[0])
            fmts.append(schema)
    blocks.append(mvcc_block(rng, 2500, 16))  # past the 32 KiB stage
    fmts.append(N.PBL_FMT_ROW)
    for i in range(0, len(blocks), 37):  # a few corrupt blocks stay failed
        b = bytearray(blocks[i])
        b[rng.randrange(len(b))] ^= 0x5A
        blocks[i] = bytes(b)
    buf, off, lens = pack(blocks)
    bf = np.array(fmts, np.uint8)
    o = oracle.decode_batch(buf, off, lens, 0, bf, flags | HIDE)
    plain = oracle.decode_batch(buf, off, lens, 0, bf, flags)
    bb = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, flags | HIDE, block_format=bf)
    g = decode(bb).to_host()
    assert_same(g, o, f"mixed hide flags={flags}")
    assert 0 < g["n_kv"] < plain["n_kv"]
    t = size_batch(bb).read_totals()
    assert int(t.n_kv) == int(o["n_kv"]) and int(t.key_bytes) == int(o["key_bytes_total"])
    assert int(t.val_bytes) == int(o["val_bytes_total"])


@pytest.mark.parametrize("every", [2, 4, 7])
def test_colblk_config3_obsolete_rows(every):
    """Config-3 blocks with every `every`-th row isObsolete (bench.py --hide):
    the pipeline's fused hide against the oracle, also when the batch carries
    the one-block-per-workgroup hints (the flag routes to the pipeline)."""
    from pebble_amd.colblk import gen_col_blocks
    buf, off, lens, n = gen_col_blocks(5 + every, 300, 32768, obsolete_every=every)
    o = oracle.transform_batch(oracle.decode_batch(buf, off, lens, N.PBL_FMT_COL_CRDB1, None, 0), 0, True)
    assert o["n_kv"] < n
    for extra in (0, N.PBL_BATCH_VARLEN, N.PBL_KERNEL_SINGLE):
        g = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_CRDB1, HIDE | extra)).to_host()
        assert_same(g, o, f"config-3 obsolete every {every} extra={extra:#x}")


@pytest.mark.parametrize("every", [2, 4])
def test_row_config2_obsolete_points(every):
    buf, off, lens, n = gen_row_blocks(9 + every, 400, 32768, 16, 16, 100, obsolete_every=every)
    g = check(buf, off, lens, 0, f"config-2 obsolete every {every}")
    assert g["n_kv"] < n
