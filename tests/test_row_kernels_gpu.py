"""The row kernels -- the staging-pool kernel (rowblk_pool.hip.h, with its
general walk and the big-block passes; PBL_KERNEL_POOL) and the two-pass form
of PBL_BATCH_VARLEN batches (rowblk_wave.hip.h: lane-per-block size walk,
bases scan, wave-per-block emit) -- against the oracle: bit-exact on every
output array, over reference blocks, synthetic configs, random and fuzzed
blocks, value prefixes, blocks past the LDS limits, the general-path fallbacks,
batches whose block shapes vary, overflowing capacities and the size pass.
(Batches whose flags need key bytes to size a block -- value prefixes --
take the pool kernel under either flag.)"""
import os
import random

import numpy as np
import pytest

import oracle
from pebble_amd import _native as N
from pebble_amd.rowblk import Writer, gen_row_blocks
from test_rowblk_gpu import GOLDEN, assert_same, pack, random_block

pytestmark = pytest.mark.gpu
KERNELS = {"pool": N.PBL_KERNEL_POOL, "wave": N.PBL_BATCH_VARLEN}


@pytest.fixture(params=sorted(KERNELS))
def kern(request):
    return KERNELS[request.param]


def check(buf, off, lens, flags=0, ctx="", kern=0):
    from pebble_amd.batch import BlockBatch, decode
    o = oracle.rowblk_decode_batch(buf, off, lens, flags)
    g = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, flags | kern)).to_host()
    assert_same(g, o, f"{ctx} kernel={kern:#x}")
    return g


def test_hamlet_and_golden(golden, kern):
    g = golden["h_no_compression"]
    blob = np.fromfile(os.path.join(GOLDEN, "h_no_compression_blocks.bin"), np.uint8)
    blob = np.concatenate([blob, np.zeros(16, np.uint8)])
    check(blob, np.array(g["block_off"], np.uint64), np.array(g["block_len"], np.uint32), 0, "hamlet", kern)
    wp = bytes.fromhex(golden["writer_with_prefix"]["block_hex"])
    wb = bytes.fromhex(golden["writer_basic"]["block_hex"])
    for flags in (0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_RAW_KEYS):
        check(*pack([wp, wb, wp]), flags, f"golden flags={flags}", kern)


@pytest.mark.parametrize("ri", [1, 2, 16, 17, 32, 64])
@pytest.mark.parametrize("kl,vl", [(16, 100), (8, 0), (64, 7), (24, 1000)])
@pytest.mark.parametrize("vp", [False, True])
def test_synthetic_batches(ri, kl, vl, vp, kern):
    for bs in (4096, 32768):
        buf, off, lens, n = gen_row_blocks(1000 + ri + kl + vl, 48, bs, ri, kl, vl, vp)
        g = check(buf, off, lens, N.PBL_ROW_VALUE_PREFIX if vp else 0, f"ri={ri} kl={kl} vl={vl} vp={vp} bs={bs}", kern)
        assert g["n_kv"] == n


def test_random_blocks(kern):
    rng = random.Random(4321)
    for flags in (0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_VALUE_PREFIX | N.PBL_ROW_NO_VALUER, N.PBL_ROW_RAW_KEYS):
        blocks = [random_block(rng)[0] for _ in range(300)]
        for align in (8, 1):
            check(*pack(blocks, align), flags, f"random flags={flags} align={align}", kern)


def test_fuzzed_blocks(kern):
    rng = random.Random(98)
    blocks = []
    for _ in range(400):
        b = bytearray(random_block(rng)[0])
        r = rng.random()
        if r < 0.3 and len(b) > 4:
            for _ in range(rng.randint(1, 4)):
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif r < 0.4:
            b = b[: rng.randint(0, len(b))]
        elif r < 0.45:
            b[-4:] = (0).to_bytes(4, "little")
        blocks.append(bytes(b))
    blocks += [b"", b"\x00", b"\x00\x00\x00\x00", Writer(16).finish()]
    for flags in (0, N.PBL_ROW_VALUE_PREFIX):
        g = check(*pack(blocks, 8), flags, f"fuzz flags={flags}", kern)
        assert g["n_bad_blocks"] > 0


@pytest.mark.parametrize("bs", [65536, 200000])
def test_blocks_past_the_limit(bs, kern):
    buf, off, lens, n = gen_row_blocks(5, 6, bs, 16, 16, 100)
    small = gen_row_blocks(6, 10, 32768, 16, 16, 100)
    blocks = [bytes(buf[o:o + l]) for o, l in zip(off, lens)] + [bytes(small[0][o:o + l]) for o, l in zip(small[1], small[2])]
    rng = random.Random(bs)
    rng.shuffle(blocks)
    check(*pack(blocks), 0, f"bs={bs}", kern)


@pytest.mark.parametrize("mix", ["zipf10", "tail8"])
def test_row_shape_mixes(mix, kern):
    """Batches whose block shapes vary inside the batch (config-2 blocks with
    Zipf blocks or short table-tail blocks interleaved), on every row kernel
    and on the default routing."""
    from pebble_amd.batch import gen_row_mix
    buf, off, lens, n = gen_row_mix(77, 600, mix)
    g = check(buf, off, lens, 0, f"mix={mix}", kern)
    assert g["n_kv"] == n and g["status_mask"] == 0
    g0 = check(buf, off, lens, 0, f"mix={mix} default", 0)
    assert g0["n_kv"] == n


def test_big_blocks_with_long_keys(kern):
    """Blocks past the 32 KiB stage whose keys outgrow the 8 KiB key buffers
    of the sizes pass's tier 1 and of the row kernel's own walk (the sizes tier
    2 and the values pass take them, with the whole 32 KiB buffer), next to big
    blocks with short keys, shared prefixes reaching deep into the long keys,
    and ordinary blocks."""
    from rowutil import make_trailer
    rng = random.Random(77)
    blocks = []
    for i in range(6):
        w = Writer(rng.choice([1, 4, 16]))
        base = bytes(rng.randrange(256) for _ in range(rng.choice([9000, 12000, 20000])))
        for k in range(8):
            key = base[: len(base) - 40] + b"%08d" % (1000 * i + k) + bytes(rng.randrange(256) for _ in range(32))
            w.add(key, make_trailer(100 + k, 1), bytes([k]) * rng.choice([100, 3000, 40000]))
        blocks.append(w.finish())
    for i in range(6):
        w = Writer(16)
        for k in range(5):
            w.add(b"short%04d-%02d" % (i, k), make_trailer(5 + k, 1), bytes([i]) * 20000)
        blocks.append(w.finish())
    small = gen_row_blocks(9, 20, 32768, 16, 16, 100)
    blocks += [bytes(small[0][o:o + l]) for o, l in zip(small[1], small[2])]
    assert sum(len(b) > 32768 for b in blocks) >= 10
    rng.shuffle(blocks)
    check(*pack(blocks), 0, "big blocks, long keys", kern)


def test_big_blocks_with_keys_near_the_slot():
    """Big blocks whose keys sit around the row kernel's slot and the sizes
    pass's 8 KiB buffer: some walked by the row kernel itself, some listed for
    the values pass, some for the sizes pass's second tier."""
    from rowutil import make_trailer
    rng = random.Random(79)
    blocks = []
    for i, kl in enumerate([3000, 5000, 6500, 7000, 7500, 7900, 8100, 8150, 8300]):
        w = Writer(rng.choice([1, 16]))
        base = bytes(rng.randrange(256) for _ in range(kl - 16))
        for k in range(3):
            w.add(base + b"%08d" % (10 * i + k), make_trailer(7 + k, 1), bytes([k + i]) * rng.choice([50, 30000]))
        blocks.append(w.finish())
    small = gen_row_blocks(10, 12, 32768, 16, 16, 100)
    blocks += [bytes(small[0][o:o + l]) for o, l in zip(small[1], small[2])]
    rng.shuffle(blocks)
    check(*pack(blocks), 0, "big blocks, keys near the slot")


def test_keys_past_the_wave_key_buffer(kern):
    """Blocks inside the 32 KiB stage whose keys outgrow the two-pass emit's
    4 KiB LDS key buffer (re-walked from global memory with the stage as the
    key buffer), shared prefixes reaching into the long keys, next to ordinary
    blocks."""
    from rowutil import make_trailer
    rng = random.Random(81)
    blocks = []
    for i, kl in enumerate([1000, 4000, 4047, 4048, 4100, 6000, 9000]):
        w = Writer(rng.choice([1, 2, 16]))
        base = bytes(rng.randrange(256) for _ in range(kl - 16))
        for k in range(3):
            w.add(base + b"%08d" % (10 * i + k), make_trailer(3 + k, 1), bytes([k + i]) * rng.choice([0, 50, 3000]))
        blocks.append(w.finish())
    small = gen_row_blocks(13, 12, 32768, 16, 16, 100)
    blocks += [bytes(small[0][o:o + l]) for o, l in zip(small[1], small[2])]
    rng.shuffle(blocks)
    check(*pack(blocks), 0, "keys past the key buffer", kern)
    check(*pack(blocks), N.PBL_ROW_RAW_KEYS, "keys past the key buffer, raw", kern)


def test_overflow_and_size_pass(kern):
    """Capacities too small: every block reports PBL_OVERFLOW with exact sizes,
    the retry decodes; the size pass alone gives the same bases and totals."""
    import torch
    from pebble_amd.batch import BlockBatch, Capacity, DecodedBatch, decode_into, decode, gen_zipf_blocks, size_batch
    buf, off, lens, n = gen_zipf_blocks(21, 64, N.PBL_FMT_ROW, 16)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, kern)
    out = DecodedBatch.allocate(64, Capacity(kv=10, key=10, val=10, rst=10), "cuda")
    decode_into(b, out)
    torch.cuda.synchronize()
    t = out.read_totals()
    assert t.status_mask & (1 << N.PBL_OVERFLOW) and t.n_kv == n
    h = decode(b, cap=Capacity(kv=10, key=10, val=10, rst=10)).to_host()
    assert h["n_kv"] == n and h["status_mask"] == 0
    s = size_batch(b)
    torch.cuda.synchronize()
    ts = s.read_totals()
    assert (ts.n_kv, ts.key_bytes, ts.val_bytes, ts.n_restarts, ts.status_mask) == \
        (h["n_kv"], h["key_bytes_total"], h["val_bytes_total"], h["n_restarts"], 0)
    assert np.array_equal(s.blk_kv_base.cpu().numpy(), h["blk_kv_base"])
    assert np.array_equal(s.blk_val_base.cpu().numpy(), h["blk_val_base"])
