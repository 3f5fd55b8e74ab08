"""Parity of the HIP row-block decoder (through the C-ABI) against the CPU
oracle: bit-exact on every array of the output contract (include/pebble_amd.h).
"""
import os
import random

import numpy as np
import pytest

import oracle
from ddutil import parse_ikeys, run_iter_cmds
from pebble_amd import _native as N
from pebble_amd.rowblk import Iter, NewIter, Transforms, Writer, gen_row_blocks, kvs_of_block, make_trailer

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ARRAYS = ["trailer", "kv_flags", "entry_off", "key_off", "val_off", "key_bytes", "val_bytes", "restarts",
          "blk_kv_base", "blk_key_base", "blk_val_base", "blk_rst_base", "blk_status"]


def gpu_decode(buf, off, lens, flags=0, cap=None):
    from pebble_amd.batch import BlockBatch, decode
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, flags)
    return decode(b, cap=cap).to_host()


def assert_same(g, o, ctx=""):
    assert g["n_kv"] == o["n_kv"], ctx
    assert g["key_bytes_total"] == o["key_bytes_total"], ctx
    assert g["val_bytes_total"] == o["val_bytes_total"], ctx
    assert g["n_restarts"] == o["n_restarts"], ctx
    assert g["status_mask"] == o["status_mask"], ctx
    assert g["n_bad_blocks"] == o["n_bad_blocks"], ctx
    for k in ARRAYS:
        a, b = g[k], o[k]
        if a is None:
            continue
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0] if a.shape == b.shape else None
            raise AssertionError(f"{ctx} array {k} differs (shape {a.shape} vs {b.shape}); first bad {bad[:10] if bad is not None else ''}")


def check(buf, off, lens, flags=0, ctx=""):
    o = oracle.rowblk_decode_batch(buf, off, lens, flags)
    g = gpu_decode(buf, off, lens, flags)
    assert_same(g, o, ctx)
    return g


def pack(blocks, align=8):
    offs, lens, pos = [], [], 0
    for bk in blocks:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        lens.append(len(bk))
        pos += len(bk)
    buf = np.zeros(pos + 16, np.uint8)
    for o, bk in zip(offs, blocks):
        buf[o:o + len(bk)] = np.frombuffer(bk, np.uint8)
    return buf, np.array(offs, np.uint64), np.array(lens, np.uint32)


def test_hamlet_sst_blocks(golden):
    g = golden["h_no_compression"]
    blob = np.fromfile(os.path.join(GOLDEN, "h_no_compression_blocks.bin"), np.uint8)
    blob = np.concatenate([blob, np.zeros(16, np.uint8)])
    r = check(blob, np.array(g["block_off"], np.uint64), np.array(g["block_len"], np.uint32), 0, "hamlet")
    kvs = []
    for b in range(len(g["block_off"])):
        kvs += kvs_of_block(r, b)
    assert [(kv.user_key.decode(), kv.value.decode()) for kv in kvs] == [tuple(x) for x in golden["hamlet_kvs"]]


def test_golden_writer_blocks(golden):
    wp = bytes.fromhex(golden["writer_with_prefix"]["block_hex"])
    wb = bytes.fromhex(golden["writer_basic"]["block_hex"])
    for flags in (0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_RAW_KEYS):
        check(*pack([wp, wb, wp]), flags, f"golden flags={flags}")


@pytest.mark.parametrize("ri", [1, 2, 3, 4])
def test_rowblk_iter_datadriven_on_gpu(golden, ri):
    # TestBlockIter2 (rowblk_iter_test.go:123-161) through rowblk.NewIter on the device
    blk = None
    for case in golden["rowblk_iter_datadriven"]:
        cmd = case["cmd"].split()
        if cmd[0] == "build":
            w = Writer(ri)
            for k, s in parse_ikeys(case["input"]):
                w.add(k, make_trailer(s, 1), b"")
            blk = w.finish()
        else:
            gsn = int(cmd[1].split("=")[1]) if len(cmd) > 1 else 0
            it = NewIter(blk, transforms=Transforms(gsn))
            assert run_iter_cmds(it, case["input"]) == case["expected"], case


@pytest.mark.parametrize("ri", [1, 2, 16, 17, 32, 64])
@pytest.mark.parametrize("kl,vl", [(16, 100), (8, 0), (64, 7), (24, 1000)])
@pytest.mark.parametrize("vp", [False, True])
def test_synthetic_batches(ri, kl, vl, vp):
    for bs in (4096, 32768):
        buf, off, lens, n = gen_row_blocks(1000 + ri + kl + vl, 48, bs, ri, kl, vl, vp)
        g = check(buf, off, lens, N.PBL_ROW_VALUE_PREFIX if vp else 0, f"ri={ri} kl={kl} vl={vl} vp={vp} bs={bs}")
        assert g["n_kv"] == n


@pytest.mark.parametrize("bs", [65536, 200000])
def test_blocks_larger_than_lds(bs):
    buf, off, lens, n = gen_row_blocks(5, 6, bs, 16, 16, 100)
    g = check(buf, off, lens, 0, f"bs={bs}")
    assert g["n_slow_blocks"] == 6 and g["n_kv"] == n


def random_block(rng: random.Random):
    ri = rng.choice([1, 2, 3, 5, 16, 33])
    w = Writer(ri)
    n = rng.randint(0, 300)
    key = b""
    vp = rng.random() < 0.5
    for i in range(n):
        keep = rng.randint(0, len(key))
        key = key[:keep] + bytes(rng.randint(97, 122) for _ in range(rng.randint(1 if i else 1, 12)))
        kind = rng.choice([0, 1, 1, 1, 2, 7, 15])
        tr = make_trailer(rng.randint(0, (1 << 56) - 1), kind)
        val = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 3, 40, 200])))
        if vp and kind == 1:
            pre = rng.choice([0x00, 0x20, 0x80, 0x81, 0x47, 0xC0])
            w.add_with_optional_value_prefix(key, tr, rng.random() < 0.2, val, len(key), True, pre, rng.random() < 0.5)
        else:
            w.add_with_optional_value_prefix(key, tr, rng.random() < 0.2, val, rng.randint(0, len(key)), False, 0,
                                             rng.random() < 0.5)
    return w.finish(), vp


def test_random_blocks_mixed_batch():
    rng = random.Random(1234)
    for flags in (0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_VALUE_PREFIX | N.PBL_ROW_NO_VALUER):
        blocks = [random_block(rng)[0] for _ in range(300)]
        for align in (8, 1):
            check(*pack(blocks, align), flags, f"random flags={flags} align={align}")


def test_corrupt_and_fuzzed_blocks():
    rng = random.Random(99)
    blocks = []
    for _ in range(400):
        blk, _vp = random_block(rng)
        b = bytearray(blk)
        r = rng.random()
        if r < 0.3 and len(b) > 4:
            for _ in range(rng.randint(1, 4)):
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif r < 0.4:
            b = b[: rng.randint(0, len(b))]
        elif r < 0.45:
            b[-4:] = (0).to_bytes(4, "little")
        elif r < 0.5:
            b[-4:] = rng.getrandbits(32).to_bytes(4, "little")
        blocks.append(bytes(b))
    blocks += [b"", b"\x00", b"\x00\x00\x00\x00", Writer(16).finish()]
    for flags in (0, N.PBL_ROW_VALUE_PREFIX):
        g = check(*pack(blocks, 8), flags, f"fuzz flags={flags}")
        assert g["n_bad_blocks"] > 0


def test_overflow_is_reported_and_retried():
    from pebble_amd.batch import BlockBatch, Capacity, DecodedBatch, decode_into, decode
    import torch
    buf, off, lens, n = gen_row_blocks(3, 16, 32768, 16, 16, 100)
    b = BlockBatch.from_host(buf, off, lens, "cuda")
    out = DecodedBatch.allocate(16, Capacity(kv=10, key=10, val=10, rst=10), "cuda")
    decode_into(b, out)
    torch.cuda.synchronize()
    t = out.read_totals()
    assert t.status_mask & (1 << N.PBL_OVERFLOW)
    assert t.n_kv == n  # sizes are exact even when nothing is written
    h = decode(b, cap=Capacity(kv=10, key=10, val=10, rst=10)).to_host()
    assert h["n_kv"] == n and h["status_mask"] == 0


def test_rebase_offset_concat():
    from pebble_amd.batch import BlockBatch, decode, rebase
    import torch
    buf, off, lens, n = gen_row_blocks(11, 8, 32768, 16, 16, 100)
    out = decode(BlockBatch.from_host(buf, off, lens, "cuda"))
    before = out.blk_kv_base[:9].clone()
    rebase(out, 1000, 2000, 3000, 4000)
    torch.cuda.synchronize()
    assert torch.equal(out.blk_kv_base[:9] - before, torch.full_like(before, 1000))


def test_device_offset_concat_matches_exclusive_prefix():
    import torch
    from pebble_amd.batch import BlockBatch, decode, offset_concat
    from pebble_amd.shard import exclusive_bases
    buf, off, lens, n = gen_row_blocks(12, 8, 32768, 16, 16, 100)
    out = decode(BlockBatch.from_host(buf, off, lens, "cuda"))
    before = torch.stack([out.blk_kv_base[:9], out.blk_key_base[:9], out.blk_val_base[:9], out.blk_rst_base[:9]]).clone()
    totals = torch.tensor([[5, 50, 500, 7], [11, 110, 1100, 13], [1, 2, 3, 4]], dtype=torch.int64, device="cuda")
    offset_concat(out, totals.reshape(-1).contiguous(), 2)
    torch.cuda.synchronize()
    after = torch.stack([out.blk_kv_base[:9], out.blk_key_base[:9], out.blk_val_base[:9], out.blk_rst_base[:9]])
    exp = exclusive_bases(totals, 2)
    assert torch.equal(after - before, exp.view(4, 1).expand(4, 9))


def test_wide_aggregates_in_lookback():
    """Blocks whose counts overflow the packed look-back word (>= 16384 KVs,
    >= 4096 restarts, >= 256 KiB of values) mixed with ordinary ones."""
    small = gen_row_blocks(5, 6, 32768, 16, 16, 100)
    many = gen_row_blocks(6, 2, 700000, 1, 16, 0)        # ~30 K KVs and restarts each
    big = gen_row_blocks(7, 2, 600000, 16, 16, 3000)      # ~590 KB of values each
    blocks = []
    for buf, off, lens, _ in (small, many, big):
        blocks += [bytes(buf[o:o + l]) for o, l in zip(off, lens)]
    order = [0, 6, 1, 8, 2, 3, 7, 4, 9, 5]
    check(*pack([blocks[i] for i in order]), 0, "wide aggregates")
