#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the pipelined row decode kernel.

Runs the PBL_STAMPS build (libpebble_amd_diag.so) on a config-2 batch and prints
per-phase median / mean / p90 shader cycles per block.  Stamps (rowblk_pipe.hip.h):
  0 parse start, 1 count pass + scan, 2 write pass, 3 parse end (published),
  4 look-back resolved (parse wave), 5 emit start, 6 per-KV arrays, 7 keys, 8 values (wave 1),
  9-11 per-emitter-wave end, 12 iteration barrier (emit side), 13 iteration
  barrier (parse side).
Read the shares, not the absolute length: the stamps themselves perturb timing.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PBL_LIB"] = os.path.join(ROOT, "pebble_amd", "libpebble_amd_diag.so")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd.batch import BlockBatch, decode  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ri = int(sys.argv[2]) if len(sys.argv) > 2 else 16
buf, off, lens, n = gen_row_blocks(42, nb, 32768, ri, 16, 100, n_threads=16)
b = BlockBatch.from_host(buf, off, lens, "cuda")
out = decode(b)
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
phases = [("parse: init+count+scan", 0, 1), ("parse: write pass", 1, 2), ("parse: buckets+publish", 2, 3),
          ("parse total", 0, 3), ("parse: look-back resolve", 3, 4), ("resolved -> emit start", 4, 5),
          ("emit: per-KV", 5, 6), ("emit: keys", 6, 7), ("emit: values (w1)", 7, 8),
          ("emit total (w1)", 5, 8), ("emit w1 end -> barrier", 8, 12), ("parse end -> barrier", 4, 13)]
print(f"blocks={nb} ri={ri} kvs={n}")
for nm, a, z in phases:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:26s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f} cycles")
for w in (9, 10, 11):
    m = (st[:, 5] > 0) & (st[:, w] > 0)
    d = (st[m, w] - st[m, 5]).astype(np.float64)
    print(f"emit wave {w - 8} start->end     median {np.median(d):9.0f} p90 {np.percentile(d, 90):9.0f}")
t0 = st[:, 0][st[:, 0] > 0]
t1 = st[:, 8][st[:, 8] > 0]
print(f"kernel span (first parse .. last emit) {t1.max() - t0.min():.0f} cycles; "
      f"{(t1.max() - t0.min()) / nb * 512:.0f} cycles per block per workgroup-slot")
# Role placement (slots 14/15: HW_ID | XCC_ID << 32 of the parse wave and emit wave 1):
# per CU, the SIMDs its parse waves ran on.
hw = st[:, 14].astype(np.uint64)
hw1 = st[:, 15].astype(np.uint64)
ok = hw != 0
simd = (hw >> np.uint64(4)) & np.uint64(3)
cu = ((hw >> np.uint64(32)) & np.uint64(15)) << np.uint64(12) | ((hw >> np.uint64(8)) & np.uint64(0x1f)) | \
     (((hw >> np.uint64(12)) & np.uint64(0xf)) << np.uint64(5))
sets = {}
for c, s in zip(cu[ok].tolist(), simd[ok].tolist()):
    sets.setdefault(c, set()).add(s)
sizes = np.bincount([len(v) for v in sets.values()], minlength=5)
print(f"CUs seen {len(sets)}; parse-wave SIMD sets per CU by size (0..4): {sizes.tolist()}")
print("parse-wave SIMD histogram:", np.bincount(simd[ok].astype(np.int64), minlength=4).tolist(),
      " emit-wave-1 SIMD histogram:", np.bincount(((hw1[hw1 != 0] >> np.uint64(4)) & np.uint64(3)).astype(np.int64),
                                                  minlength=4).tolist())
