#!/usr/bin/env python3
"""Phase cycles per block of the snappy kernels (diagnostic build with
-DPBL_SNAP_STAMPS, loaded through PBL_LIB): staging / bitmap load, parse,
copy resolution, literals, ordered copies, and the round and copy-group
counts, medians over a config-2-shaped batch or, with CORPUS=words, the
text corpus of scripts/prof_zstd.py (512 distinct blocks cycled)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.physical import PhysBatch, decompress  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
if os.environ.get("CORPUS") == "words":
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
    words = [bytes(alpha[rng.integers(0, len(alpha), int(k))]) + b" " for k in rng.integers(2, 9, 512)]
    raw = [b"".join(words[i] for i in rng.integers(0, 512, 8000))[:32768] for _ in range(512)]
    comp = [pa.Codec("snappy").compress(raw[i % 512], asbytes=True) for i in range(nb)]
else:
    buf, off, lens, _ = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
    comp = [pa.Codec("snappy").compress(buf[int(o):int(o) + int(ln)].tobytes(), asbytes=True)
            for o, ln in zip(off, lens)]
cl = np.array([len(x) for x in comp], np.uint32)
coff = np.zeros(nb, np.uint64)
coff[1:] = np.cumsum((cl.astype(np.uint64) + 5 + 7) // 8 * 8)[:-1]
cbuf = np.zeros(int(coff[-1]) + int(cl[-1]) + 32, np.uint8)
for i, x in enumerate(comp):
    cbuf[int(coff[i]):int(coff[i]) + len(x)] = np.frombuffer(x, np.uint8)
    cbuf[int(coff[i]) + len(x)] = 1
L = N.lib()
f = L.pbl_diag_snap_stamps
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
pb = PhysBatch.from_host(cbuf, coff, cl)
decompress(pb)
torch.cuda.synchronize()
assert f(None, 0, 1) == 0
bb, st = decompress(pb)
torch.cuda.synchronize()
assert not st.any()
h = np.zeros(65536 * 8, np.uint64)
assert f(h.ctypes.data, 65536 * 8, 0) == 0
h = h.reshape(65536, 8)[:nb].astype(np.float64)
names = ["stage", "parse", "literals", "copies", "rounds", "groups", "resolve"]
for k, nm in enumerate(names):
    print(f"{nm:10s} median {np.median(h[:, k]):10.0f} mean {h[:, k].mean():10.0f} p90 {np.percentile(h[:, k], 90):10.0f}")
