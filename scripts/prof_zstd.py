#!/usr/bin/env python3
"""Profiling driver: a text-like corpus (bench_physical.py's kind, 512 distinct
blocks cycled) compressed with zstd level 3 (ratio ~2.66) or, with
CODEC=snappy, snappy (~1.95), decompressed `iters` times (for rocprofv3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv += [] if len(sys.argv) > 1 else ["8192"]
import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

from pebble_amd.physical import PhysBatch, decompress  # noqa: E402

nb = int(sys.argv[1])
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
level = int(os.environ.get("ZSTD_LEVEL", "3"))
rng = np.random.default_rng(5)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
words = [bytes(alpha[rng.integers(0, len(alpha), int(k))]) + b" " for k in rng.integers(2, 9, 512)]
codec = os.environ.get("CODEC", "zstd")
c = pa.Codec("zstd", compression_level=level) if codec == "zstd" else pa.Codec("snappy")


def uvarint(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


raw = [b"".join(words[i] for i in rng.integers(0, 512, 8000))[:32768] for _ in range(512)]
comp = [(uvarint(len(b)) if codec == "zstd" else b"") + c.compress(b, asbytes=True) for b in raw]
cl = np.array([len(comp[i % len(comp)]) for i in range(nb)], np.uint32)
coff = np.zeros(nb, np.uint64)
coff[1:] = np.cumsum((cl.astype(np.uint64) + 5 + 7) // 8 * 8)[:-1]
cbuf = np.zeros(int(coff[-1]) + int(cl[-1]) + 32, np.uint8)
for i in range(nb):
    x = comp[i % len(comp)]
    cbuf[int(coff[i]):int(coff[i]) + len(x)] = np.frombuffer(x, np.uint8)
    cbuf[int(coff[i]) + len(x)] = 7 if codec == "zstd" else 1
pb = PhysBatch.from_host(cbuf, coff, cl)
for _ in range(iters):
    bb, st = decompress(pb)
torch.cuda.synchronize()
assert not st.any()
print(f"{nb} blocks, ratio {sum(len(r) for r in raw) / sum(len(x) for x in comp):.2f}, nseq-ish n/a")
