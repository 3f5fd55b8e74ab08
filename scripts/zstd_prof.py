#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of zstd_kernel (PBL_ZSTD_STAMPS build loaded via
PBL_LIB=<diag .so>) on the text-like corpus of bench_physical.py (level 3).
Phases (summed over blocks, then per block): 0 literals (header, Huffman table,
streams), 1 sequence tables, 2 sequence decode (lane 0), 3 sequence execution,
5 input staging, 6 output write, 7 whole block."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], sys.argv[1] if len(sys.argv) > 1 else "8192", "1", "zstd"]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pyarrow as pa  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.physical import PhysBatch, decompress  # noqa: E402

nb = int(sys.argv[1])
rng = np.random.default_rng(5)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
words = [bytes(alpha[rng.integers(0, len(alpha), int(k))]) + b" " for k in rng.integers(2, 9, 512)]
raw = []
for _ in range(256):
    ids = rng.integers(0, 512, 8000)
    raw.append(b"".join(words[i] for i in ids)[:32768])
c = pa.Codec("zstd", compression_level=3)


def uvarint(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


comp = [uvarint(len(b)) + c.compress(b, asbytes=True) for b in raw]
cl = np.array([len(comp[i % 256]) for i in range(nb)], np.uint32)
coff = np.zeros(nb, np.uint64)
coff[1:] = np.cumsum((cl.astype(np.uint64) + 5 + 7) // 8 * 8)[:-1]
cbuf = np.zeros(int(coff[-1]) + int(cl[-1]) + 32, np.uint8)
for i in range(nb):
    x = comp[i % 256]
    cbuf[int(coff[i]):int(coff[i]) + len(x)] = np.frombuffer(x, np.uint8)
    cbuf[int(coff[i]) + len(x)] = 7
pb = PhysBatch.from_host(cbuf, coff, cl)
lib = N.lib()
fn = lib.pbl_diag_zstd_prof
fn.argtypes = [ctypes.c_void_p]
acc = (ctypes.c_ulonglong * 8)()
bb, st = decompress(pb)
torch.cuda.synchronize()
fn(acc)  # clear (the first pass includes the warm-up)
bb, st = decompress(pb)
torch.cuda.synchronize()
assert not st.any()
fn(acc)
names = {0: "literals", 1: "seq tables", 2: "seq decode (lane 0)", 3: "seq execution", 5: "stage in", 6: "write out",
         7: "whole block"}
print(f"{nb} blocks, ratio {sum(len(r) for r in raw) / sum(len(x) for x in comp):.2f}")
for k, nm in names.items():
    print(f"{nm:22s} {acc[k] / nb:12.0f} cycles/block")
