#!/usr/bin/env python3
"""Throughput of the physical-block step on config-2-shaped
data: 64 Ki x 32 KiB row blocks with 5-byte trailers.  The trailers' checksums
are produced by the device itself (a first verify pass reports `computed`,
which is written into the trailers; the timed passes then verify them all OK).
Snappy: the same blocks compressed on the host (pyarrow), decompressed on the
device; also a text-like corpus (~2x for snappy) and zstd (level 3, Pebble's
uvarint length prefix) and MinLZ (indicator 8, Snappy form) on both; every
block distinct.  Prints one JSON line.
Usage: bench_physical.py [n_blocks] [reps] [codecs, e.g. snappy,zstd]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.physical import PhysBatch, decompress, verify_checksums  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
buf, off, lens, _ = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
stride = 32768 + 8
phys = np.zeros(nb * stride + 16, np.uint8)
pv = phys[: nb * stride].reshape(nb, stride)
pv[:, :32768] = buf[: nb * 32768].reshape(nb, 32768)
poff = np.arange(nb, dtype=np.uint64) * stride
res = {"blocks": nb, "block_bytes": int(lens.sum())}


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


for name, ct in (("crc32c", N.PBL_CHECKSUM_CRC32C), ("xxhash64", N.PBL_CHECKSUM_XXHASH64)):
    pb = PhysBatch.from_host(phys, poff, lens)
    _, comp = verify_checksums(pb, ct)
    # write the device-computed checksums into the trailers (indicator 0 = none)
    host = pb.bytes.cpu().numpy()
    for i in range(nb):
        t = int(poff[i]) + int(lens[i])
        host[t + 1:t + 5] = np.frombuffer(int(comp[i]).to_bytes(4, "little"), np.uint8)
    pb = PhysBatch(torch.from_numpy(host).cuda(), pb.block_off, pb.block_len)
    st, _ = verify_checksums(pb, ct)
    assert not st.any()
    from pebble_amd.batch import _stream_handle
    import ctypes
    s_t = torch.empty(nb, dtype=torch.int32, device="cuda")
    c = pb.c_struct()
    sec = timed(lambda: N.lib().pbl_verify_checksums(ctypes.byref(c), ct, ctypes.c_void_p(s_t.data_ptr()), None,
                                                      _stream_handle(None)))
    res[name] = {"GB_per_s": round((int(lens.sum()) + nb) / sec / 1e9, 1), "ms": round(sec * 1e3, 3)}

import ctypes  # noqa: E402

import pyarrow as pa  # noqa: E402

from pebble_amd.batch import _stream_handle  # noqa: E402


def uvarint(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def words_blocks(n_distinct=256, vocab=512, seed=5):
    """Text-like 32 KiB blocks (a 512-word vocabulary: snappy ~2x, zstd ~3x),
    every block distinct."""
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
    wl = rng.integers(2, 9, vocab)
    W = np.zeros((vocab, 9), np.uint8)
    for i in range(vocab):
        W[i, :wl[i]] = alpha[rng.integers(0, len(alpha), int(wl[i]))]
        W[i, wl[i]] = ord(" ")
    keep = np.arange(9)[None, :] <= wl[:, None]
    ids = rng.integers(0, vocab, 12_000_000)
    text = W[ids][keep[ids]]  # ~66 MB of words; block i = a 32 KiB window at a random offset
    stride = (len(text) - 32768) // n_distinct  # distinct offsets, in random order
    starts = rng.permutation(np.arange(n_distinct) * stride + rng.integers(0, stride, n_distinct))
    return [text[a:a + 32768].tobytes() for a in starts]


def codec_run(raw_blocks, codec, n):
    """Compress the distinct raw blocks (zstd with Pebble's uvarint prefix),
    lay out n physical blocks cycling through them, decompress on the device
    (checked), time pbl_decompress_blocks."""
    # minlz: blocks with the MinLZ indicator (8) in the Snappy form, the form
    # minlz.Decode is pinned for (internal/compression/minlz_test.go:31-36);
    # the native MinLZ form is opt-in and unpinned (include/pebble_amd.h)
    ind = {"snappy": 1, "minlz": 8, "zstd": 7}[codec]
    snappy_like = codec in ("snappy", "minlz")
    c = pa.Codec("snappy") if snappy_like else pa.Codec("zstd", compression_level=3)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(16) as ex:
        comp = list(ex.map(lambda b: c.compress(b, asbytes=True) if snappy_like
                           else uvarint(len(b)) + c.compress(b, asbytes=True), raw_blocks))
    k = len(comp)
    cl = np.array([len(comp[i % k]) for i in range(n)], np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum((cl.astype(np.uint64) + 5 + 7) // 8 * 8)[:-1]
    cbuf = np.zeros(int(coff[-1]) + int(cl[-1]) + 32, np.uint8)
    for i in range(n):
        x = comp[i % k]
        cbuf[int(coff[i]):int(coff[i]) + len(x)] = np.frombuffer(x, np.uint8)
        cbuf[int(coff[i]) + len(x)] = ind
    pb = PhysBatch.from_host(cbuf, coff, cl)
    bb, st = decompress(pb)
    raw_total = sum(len(raw_blocks[i % k]) for i in range(n))
    assert not st.any() and int(bb.block_len.to(torch.int64).sum()) == raw_total, (codec, st[:8])
    out = bb.blocks.cpu().numpy()
    bo, bl = bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i in list(range(min(n, 64))) + [n - 1]:
        assert out[bo[i]:bo[i] + bl[i]].tobytes() == raw_blocks[i % k], (codec, i)
    cs = pb.c_struct()
    o_len = torch.empty(n, dtype=torch.int32, device="cuda")
    o_st = torch.empty(n, dtype=torch.int32, device="cuda")
    cap = bb.block_len.clone()
    sec = timed(lambda: N.lib().pbl_decompress_blocks(ctypes.byref(cs), ctypes.c_void_p(bb.blocks.data_ptr()),
                                                      ctypes.c_void_p(bb.block_off.data_ptr()),
                                                      ctypes.c_void_p(cap.data_ptr()),
                                                      ctypes.c_void_p(o_len.data_ptr()),
                                                      ctypes.c_void_p(o_st.data_ptr()), _stream_handle(None)))
    return {"decoded_GB_per_s": round(raw_total / sec / 1e9, 1), "ms": round(sec * 1e3, 3),
            "decoded_bytes": raw_total, "compressed_bytes": int(cl.sum()),
            "ratio": round(raw_total / float(cl.sum()), 2), "distinct_blocks": k}


cfg2 = [buf[int(o):int(o) + int(ln)].tobytes() for o, ln in zip(off, lens)]
codecs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["snappy", "minlz", "zstd"]
words = words_blocks(nb)
for codec in codecs:
    # config-2 blocks (random values: ratio ~1.0) and text-like blocks (ratio ~2-3), all distinct
    res[codec] = codec_run(cfg2, codec, nb)
    res[codec + "_words"] = codec_run(words, codec, nb)
print(json.dumps(res), flush=True)
