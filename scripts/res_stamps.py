#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of rowblk_res_kernel (PBL_STAMPS build,
PBL_LIB=<diag .so>) on a config-2 batch.  Stamps (rowblk_res.hip.h): 0 loop top
(the block's registers awaited), 1 staged (registers -> LDS), 2 walk + scan +
publish (look-back windows issued), 3 metadata, 4 look-back resolved, 5 keys /
per-KV arrays / restarts, 6 values.  Read the shares; the stamps perturb
timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.batch import BlockBatch, decode  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
buf, off, lens, n = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, N.PBL_KERNEL_RES)
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
phases = [("registers -> stage", 0, 1), ("walk + scan + publish", 1, 2), ("metadata", 2, 3),
          ("look-back finish", 3, 4), ("keys + per-KV", 4, 5), ("values", 5, 6), ("block total", 0, 6)]
for nm, a, z in phases:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:28s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f} cycles")
t0, t6 = st[:, 0][st[:, 0] > 0], st[:, 6][st[:, 6] > 0]
print(f"kernel span {t6.max() - t0.min():.0f} cycles; blocks per CU {nb / 256:.0f}; "
      f"cycles per block per CU {(t6.max() - t0.min()) / (nb / 256):.0f}")
