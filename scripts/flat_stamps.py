#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of rowblk_flat_kernel or (argument `run`)
rowblk_run_kernel (PBL_STAMPS build, libpebble_amd_diag.so) on a config-2
batch.  Stamps (rowblk_flat.hip.h): 0 block start (ticket taken), 1 staged, 2
pass 1 + publish, 3 pass 2 (metadata), 4 look-back resolved, 5 emit done;
(rowblk_run.hip.h): 0 start, 1 staged, 2 count walk + publish, 3 look-back
resolved, 4 emit done.  Read the shares; the stamps perturb timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PBL_LIB", os.path.join(ROOT, "pebble_amd", "libpebble_amd_diag.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.batch import BlockBatch, decode  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
run = len(sys.argv) > 2 and sys.argv[2] == "run"
buf, off, lens, n = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, N.PBL_KERNEL_RUN if run else N.PBL_KERNEL_FLAT)
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
phases = [("stage (DMA round trip)", 0, 1), ("pass 1 + publish", 1, 2), ("pass 2 (metadata)", 2, 3),
          ("look-back finish", 3, 4), ("emit", 4, 5), ("block total", 0, 5)]
last = 5
if run:
    phases = [("stage (DMA round trip)", 0, 1), ("count walk + publish", 1, 2), ("look-back finish", 2, 3),
              ("emit (run-major)", 3, 4), ("block total", 0, 4)]
    last = 4
for nm, a, z in phases:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:24s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f} cycles")
# gap between a wave's blocks (ticket atomic + descriptor reads): next start - this end, same wave unknown:
t0, t5 = st[:, 0][st[:, 0] > 0], st[:, last][st[:, last] > 0]
print(f"kernel span {t5.max() - t0.min():.0f} cycles; per block per wave-slot "
      f"{(t5.max() - t0.min()) / nb * 1024:.0f}")
