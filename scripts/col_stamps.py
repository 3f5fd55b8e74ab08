#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of the pipelined colblk kernel (PBL_STAMPS build).
Stamps: 0 parse start, 1 header parsed, 2 parse end (published), 3 emit start,
4 look-back resolved, 5 per-row arrays, 6 keys, 7 values."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PBL_LIB"] = os.path.join(ROOT, "pebble_amd", "libpebble_amd_diag.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.batch import BlockBatch, decode  # noqa: E402
from pebble_amd.colblk import gen_col_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
if len(sys.argv) > 2 and sys.argv[2] == "zipf":
    # config 5, colblk DefaultKeySchema (bench.py --workload zipf --zipf-format col)
    from pebble_amd.batch import gen_zipf_blocks
    buf, off, lens, n = gen_zipf_blocks(42, nb, N.PBL_FMT_COL_DEFAULT, 16, 32768, n_threads=16)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_DEFAULT, 0)
    print("blocks: len median", np.median(lens), "p99", np.percentile(lens, 99), "max", lens.max(), "kvs", n)
else:
    buf, off, lens, n = gen_col_blocks(42, nb, 32768, n_threads=16)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_CRDB1, 0)
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
for nm, a, z in [("parse: header", 0, 1), ("parse: rows + publish", 1, 2), ("parse total", 0, 2),
                 ("parse end -> emit start", 2, 3), ("emit: look-back", 3, 4), ("emit: per-row", 4, 5),
                 ("emit: keys", 5, 6), ("emit: values", 6, 7), ("emit total", 3, 7)]:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:24s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f} cycles")
r = st[:, 10]
sp = st[:, 11]
tot = st[:, 7] - st[:, 0]
m = (st[:, 0] > 0) & (st[:, 7] > 0)
if m.any():
    print("per-block parse start -> values end: median", np.median(tot[m]), "p99", np.percentile(tot[m], 99),
          "max", tot[m].max())
print("look-back rounds: median", np.median(r), "mean", r.mean(), "max", r.max(), "| spins: median", np.median(sp),
      "mean", sp.mean(), "p90", np.percentile(sp, 90))
