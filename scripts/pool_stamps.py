#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of rowblk_pool_kernel (PBL_STAMPS build,
PBL_LIB=<diag .so>) on a config-2 batch.  Stamps (rowblk_pool.hip.h): 8
acquire start, 0 stage acquired + ticket, 1 descriptor read, 2 staged (DMA
landed), 3 walk + scan + publish, 4 metadata + value buckets, 5 look-back
resolved, 6 keys / per-KV arrays written (and the stage released, unless
PBL_POOL_EARLY released it at 4), 7 values done.
Read the shares; the stamps perturb timing."""
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
wl = os.environ.get("WORKLOAD", "row")  # row (config 2) or zipf:RI (config 5, row format)
if wl.startswith("zipf"):
    from pebble_amd.batch import gen_zipf_blocks
    buf, off, lens, n = gen_zipf_blocks(42, nb, N.PBL_FMT_ROW, int(wl.split(":")[1]), 32768, n_threads=16)
else:
    buf, off, lens, n = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, N.PBL_KERNEL_POOL)
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
phases = [("acquire stage + ticket", 8, 0), ("descriptor", 0, 1), ("stage (DMA round trip)", 1, 2),
          ("walk + scan + publish", 2, 3), ("metadata + buckets", 3, 4), ("look-back finish", 4, 5),
          ("keys + per-KV", 5, 6), ("values (global)", 6, 7), ("stage held (keys from the stage)", 0, 6),
          ("stage held (PBL_POOL_EARLY)", 0, 4), ("block total", 8, 7)]
for nm, a, z in phases:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:28s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f} cycles")
t0, t7 = st[:, 8][st[:, 8] > 0], st[:, 7][st[:, 7] > 0]
print(f"kernel span {t7.max() - t0.min():.0f} cycles; blocks per CU {nb / 256:.0f}; "
      f"cycles per block per CU {(t7.max() - t0.min()) / (nb / 256):.0f}")
