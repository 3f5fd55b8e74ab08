"""Mixed row + colblk batches (config 4, block_format[]): the format split into
two ascending id lists, the colblk sizes, the row kernel over the row ids and
the colblk pipeline over the colblk ids, one look-back over the batch order,
against the oracle, bit-exact on every output array."""
import random

import numpy as np
import pytest

import oracle
from colutil import build_block, random_rows
from pebble_amd import _native as N
from pebble_amd.colblk import SCHEMA_DEFAULT, gen_col_blocks
from pebble_amd.rowblk import gen_row_blocks
from test_rowblk_gpu import assert_same, pack

pytestmark = pytest.mark.gpu


def gpu(buf, off, lens, bf, flags=0, cap=None, exact=False):
    from pebble_amd.batch import BlockBatch, decode
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, flags, block_format=bf)
    return decode(b, cap=cap, exact=exact).to_host()


def check(blocks, fmts, align=8, ctx="", **kw):
    buf, off, lens = pack(blocks, align)
    bf = np.array(fmts, np.uint8)
    o = oracle.decode_batch(buf, off, lens, N.PBL_FMT_ROW, bf)
    g = gpu(buf, off, lens, bf, **kw)
    assert_same(g, o, ctx)
    return g


def pool(seed, n_row, n_col, size=8192):
    rb, ro, rl, _ = gen_row_blocks(seed, n_row, size, 16, 16, 100)
    cb, co, cl, _ = gen_col_blocks(seed, n_col, size)
    rows = [bytes(rb[ro[i]:ro[i] + rl[i]]) for i in range(n_row)]
    cols = [bytes(cb[co[i]:co[i] + cl[i]]) for i in range(n_col)]
    return rows, cols


def test_mixed_shapes():
    rows, cols = pool(1, 40, 40)
    rng = random.Random(2)
    dflt = build_block(SCHEMA_DEFAULT, random_rows(rng, SCHEMA_DEFAULT, 150))[0]
    R, C, D = N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1, N.PBL_FMT_COL_DEFAULT
    cases = {
        "interleaved": ([x for p in zip(rows, cols) for x in p], [R, C] * 40),
        "all_row": (rows, [R] * 40),
        "all_col": (cols, [C] * 40),
        "one_row": (cols[:20] + rows[:1] + cols[20:], [C] * 20 + [R] + [C] * 20),
        "one_col": (rows[:30] + cols[:1], [R] * 30 + [C]),
        "runs": (rows[:10] + cols[:25] + [dflt] + rows[10:], [R] * 10 + [C] * 25 + [D] + [R] * 30),
    }
    for name, (blocks, fmts) in cases.items():
        for align in (8, 1):
            check(blocks, fmts, align, name)


def test_mixed_random_across_split_chunks():
    """> 4096 blocks: the format split spans several chunks."""
    rows, cols = pool(3, 64, 64, 4096)
    rng = random.Random(4)
    blocks, fmts = [], []
    for _ in range(9000):
        if rng.random() < 0.45:
            blocks.append(rng.choice(rows)); fmts.append(N.PBL_FMT_ROW)
        else:
            blocks.append(rng.choice(cols)); fmts.append(N.PBL_FMT_COL_CRDB1)
    g = check(blocks, fmts, 8, "random9000")
    assert g["status_mask"] == 0


def test_mixed_big_and_corrupt_blocks():
    """Row blocks past the LDS stage (the big-block passes must skip colblk
    blocks), colblk blocks past the head stage, corrupt blocks of both kinds."""
    rows, cols = pool(5, 8, 8)
    big_row = bytes(gen_row_blocks(6, 1, 131072, 16, 16, 100)[0][:131072])
    rng = random.Random(7)
    big_col = build_block(SCHEMA_DEFAULT, random_rows(rng, SCHEMA_DEFAULT, 30, key_len=(1000, 1500), shared=900,
                                                      val_len=(0, 8)))[0]
    bad_row = rows[0][:100]
    bad_col = bytearray(cols[0]); bad_col[5] ^= 0xff
    blocks = rows[:4] + [big_row] + cols[:4] + [big_col, bad_row, bytes(bad_col)] + rows[4:] + cols[4:] + [big_row]
    R, C, D = N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1, N.PBL_FMT_COL_DEFAULT
    fmts = [R] * 4 + [R] + [C] * 4 + [D, R, C] + [R] * 4 + [C] * 4 + [R]
    g = check(blocks, fmts, 8, "big+corrupt")
    assert g["n_bad_blocks"] >= 1



def test_mixed_big_blocks_with_long_keys():
    """Big row blocks whose keys outgrow the big-block passes' 8 KiB key buffer
    in a mixed batch: the sizes pass lists them for its second tier (the redo
    list has its own workspace area, past the format split's ids, which the
    row and colblk kernels read after it)."""
    from pebble_amd.rowblk import Writer, make_trailer
    rng = random.Random(78)
    rows, cols = pool(8, 12, 12)
    big = []
    for i in range(4):
        w = Writer(rng.choice([1, 16]))
        base = bytes(rng.randrange(256) for _ in range(rng.choice([9000, 20000])))
        for k in range(6):
            w.add(base + b"%08d" % (100 * i + k), make_trailer(10 + k, 1), bytes([k]) * rng.choice([100, 30000]))
        big.append(w.finish())
    assert all(len(b) > 32768 for b in big)
    R, C = N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1
    blocks = rows[:6] + [big[0]] + cols[:6] + [big[1], big[2]] + rows[6:] + cols[6:] + [big[3]]
    fmts = [R] * 6 + [R] + [C] * 6 + [R, R] + [R] * 6 + [C] * 6 + [R]
    check(blocks, fmts, 8, "big long keys")

def test_mixed_overflow_retry_and_size_pass():
    from pebble_amd.batch import Capacity
    rows, cols = pool(8, 20, 20)
    blocks = [x for p in zip(rows, cols) for x in p]
    fmts = [N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1] * 20
    check(blocks, fmts, 8, "overflow", cap=Capacity(kv=10, key=10, val=10, rst=10))
    check(blocks, fmts, 8, "exact", exact=True)


def _big_row_block(rng, n=6, vlen=9000):
    from pebble_amd.rowblk import Writer, make_trailer
    w = Writer(rng.choice([1, 4, 16]))
    for k in range(n):
        w.add(b"key%06d" % k, make_trailer(10 + k, 1), bytes([k]) * vlen)
    blk = w.finish()
    assert len(blk) > 32768
    return blk


def test_big_row_blocks_failing_init_checks():
    """Row blocks past the 32 KiB stage that fail rowblk.Iter.Init's checks
    (rowblk_iter.go:248-256, readFirstKey :418-485): zero restarts, a restart
    table larger than the block, a first entry with shared != 0, a first key
    shorter than 8 bytes.  The sizes pass publishes their status and a zero
    aggregate; every later block is placed after them.  Row and mixed batches."""
    rng = random.Random(91)
    rows, cols = pool(9, 6, 6)
    good = [_big_row_block(rng) for _ in range(3)]
    bad = []
    b = bytearray(_big_row_block(rng)); b[-4:] = (0).to_bytes(4, "little"); bad.append(bytes(b))       # no restarts
    b = bytearray(_big_row_block(rng)); b[-4:] = (1 << 20).to_bytes(4, "little"); bad.append(bytes(b))  # table > block
    b = bytearray(_big_row_block(rng)); b[0] = 3; bad.append(bytes(b))                                  # shared != 0
    b = bytearray(_big_row_block(rng)); b[1] = 4; bad.append(bytes(b))                                  # key < 8 bytes
    b = bytearray(_big_row_block(rng)); b[-4:] = (0x80000001).to_bytes(4, "little"); bad.append(bytes(b))  # bit 31 count
    R, C = N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1
    blocks = [good[0]] + bad[:2] + rows[:3] + [good[1]] + bad[2:] + rows[3:] + [good[2]]
    buf, off, lens = pack(blocks)
    o = oracle.decode_batch(buf, off, lens, N.PBL_FMT_ROW)
    assert o["n_bad_blocks"] == len(bad)
    for flags in (0, N.PBL_ROW_HIDE_OBSOLETE):
        assert_same(gpu(buf, off, lens, None, flags), oracle.decode_batch(buf, off, lens, N.PBL_FMT_ROW, None, flags),
                    f"row batch flags={flags}")
    mixed = [good[0], cols[0]] + bad[:2] + [cols[1]] + rows[:3] + [good[1]] + bad[2:] + cols[2:] + [good[2]]
    fm = [R, C, R, R, C] + [R] * 3 + [R] + [R] * len(bad[2:]) + [C] * 4 + [R]
    g = check(mixed, fm, 8, "mixed big bad")
    assert g["n_bad_blocks"] == len(bad)
    check(mixed, fm, 8, "mixed big bad exact", exact=True)
