"""blockiter.SyntheticSeqNum fused into the decode (pbl_block_batch.
synthetic_seq_num): a batch decoded with the field set
equals the oracle's decode followed by its SetSeqNum transform
(oracle.transform_batch, rowblk_iter.go:1168-1191; data_block.go:1693-1695),
bit-exact on every array -- row batches on every row kernel (the pool default, the
pipeline, one-block-per-workgroup; blocks past the LDS stage on the slow walk; invalid
keys keep the Invalid trailer; corrupt blocks), colblk batches of both
schemas, a mixed batch and raw-key batches (no seqnums)."""
import ctypes
import random

import numpy as np
import pytest

import oracle
from colutil import build_block, random_rows
from pebble_amd import _native as N
from pebble_amd.batch import BlockBatch, decode
from pebble_amd.colblk import SCHEMA_CRDB1, SCHEMA_DEFAULT
from pebble_amd.rowblk import Writer, gen_row_blocks, make_trailer
from test_baseline_configs_gpu import varint_blocks
from test_rowblk_gpu import assert_same, pack, random_block

pytestmark = pytest.mark.gpu
SEQS = [1, 77, (1 << 56) - 1]


def fused(buf, off, lens, fmt, seq, flags=0, block_fmt=None):
    bb = BlockBatch.from_host(buf, off, lens, "cuda", fmt, flags, block_format=block_fmt)
    bb.synthetic_seq_num = seq
    g = decode(bb).to_host()
    o = oracle.transform_batch(oracle.decode_batch(buf, off, lens, fmt, block_fmt, flags & 0xFF), seq, False, b"", b"",
                               0, src=(buf, off, lens, fmt, block_fmt, flags & 0xFF))
    return g, o


def big_row_blocks(rng):
    out = []
    for vl in (70_000, 140_000):  # past the LDS stage: the slow walk
        w = Writer(4)
        for i in range(6):
            w.add(b"big%03d" % i, make_trailer(i + 1, 1), bytes([i]) * (vl if i == 2 else 50))
        out.append(w.finish())
    return out


@pytest.mark.parametrize("kernel", [0])
@pytest.mark.parametrize("seq", SEQS)
def test_row_batches(kernel, seq):
    rng = random.Random(seq % 1000 + kernel)
    blocks = [random_block(rng)[0] for _ in range(200)] + big_row_blocks(rng) + varint_blocks()
    for i in range(0, 200, 17):
        b = bytearray(blocks[i])
        if len(b) > 8:
            b[rng.randrange(len(b))] ^= 0x41  # corrupt some
            blocks[i] = bytes(b)
    for flags in (0, N.PBL_ROW_VALUE_PREFIX):
        g, o = fused(*pack(blocks), N.PBL_FMT_ROW, seq, flags | kernel)
        assert_same(g, o, f"row seq={seq} kernel={kernel:#x} flags={flags}")


def test_config2_shaped_and_raw_keys():
    buf, off, lens, _n = gen_row_blocks(3, 2048, 32768, 16, 16, 100, n_threads=8)
    g, o = fused(buf, off, lens, N.PBL_FMT_ROW, 4242)
    assert_same(g, o, "config-2 shaped")
    assert (g["trailer"] >> 8 == 4242).all()
    # raw keys (metadata blocks): no sequence numbers to rewrite
    rng = random.Random(5)
    blocks = [random_block(rng)[0] for _ in range(50)]
    buf, off, lens = pack(blocks)
    bb = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, N.PBL_ROW_RAW_KEYS)
    plain = decode(bb).to_host()
    bb.synthetic_seq_num = 99
    assert_same(decode(bb).to_host(), plain, "raw keys")


@pytest.mark.parametrize("schema", [SCHEMA_DEFAULT, SCHEMA_CRDB1])
def test_colblk_batches(schema):
    rng = random.Random(schema)
    blocks = []
    for _ in range(60):
        rows = random_rows(rng, schema, rng.choice([1, 5, 17, 100, 300]), shared=rng.choice([0, 3]),
                           val_len=(0, rng.choice([3, 50])))
        blocks.append(build_block(schema, rows, rng.choice([1, 4, 16]))[0])
    for seq in SEQS:
        g, o = fused(*pack(blocks), schema, seq)
        assert_same(g, o, f"colblk schema={schema} seq={seq}")


def test_mixed_batch():
    rng = random.Random(11)
    blocks, fmts = [], []
    for i in range(120):
        if i % 2:
            rows = random_rows(rng, SCHEMA_CRDB1, rng.choice([5, 60]), shared=0, val_len=(0, 20))
            blocks.append(build_block(SCHEMA_CRDB1, rows, 16)[0])
            fmts.append(SCHEMA_CRDB1)
        else:
            blocks.append(random_block(rng)[0])
            fmts.append(N.PBL_FMT_ROW)
    buf, off, lens = pack(blocks)
    g, o = fused(buf, off, lens, N.PBL_FMT_ROW, 31337, block_fmt=np.array(fmts, np.uint8))
    assert_same(g, o, "mixed")


def test_seqnum_out_of_range_is_invalid_arg():
    buf, off, lens = pack([random_block(random.Random(1))[0]])
    bb = BlockBatch.from_host(buf, off, lens, "cuda")
    bb.synthetic_seq_num = 1 << 56
    from pebble_amd.batch import Capacity, DecodedBatch
    out = DecodedBatch.allocate(1, Capacity(1000, 10000, 100000, 1000), "cuda")
    assert N.lib().pbl_decode_batch(ctypes.byref(bb.c_struct()), ctypes.byref(out.c_struct()), None) == \
        N.PBL_INVALID_ARG
