#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the row decode kernel.

Runs the PBL_STAMPS build (libpebble_amd_diag.so) on a config-2 batch and
prints, per phase, the median / mean shader cycles per block.  Read the shares,
not the absolute length: the stamps themselves perturb timing.
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
ws_state = 256 + 9 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
phases = [("load+init", 0, 1), ("P1 run walk", 1, 2), ("P1 scan", 2, 3), ("vprefix P2/P4", 3, 4),
          ("look-back (w0)", 4, 9), ("P2 expand (w1-3)", 4, 10), ("join barrier", 4, 5),
          ("per-KV out", 5, 6), ("keys", 6, 7), ("values", 7, 8)]
print(f"blocks={nb} ri={ri} kvs={n}")
for nm, a, z in phases:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:20s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f} cycles")
tot = (st[:, 8] - st[:, 0]).astype(np.float64)
print(f"total per block: median {np.median(tot):.0f} mean {np.mean(tot):.0f} cycles")
