#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of the wave-per-block colblk kernel
(colblk_wave.hip.h, PBL_STAMPS build) on config 5's colblk batch.
Stamps: 0 ticket, 1 staged, 2 rows counted, 3 look-back resolved,
4 block metadata written, 5 per-row arrays, 6 keys, 7 values."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PBL_LIB"] = os.path.join(ROOT, "pebble_amd", "libpebble_amd_diag.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.batch import BlockBatch, decode, gen_zipf_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
buf, off, lens, n = gen_zipf_blocks(42, nb, N.PBL_FMT_COL_DEFAULT, 16, 32768, n_threads=16)
b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_DEFAULT, 0)
print("blocks: len median", np.median(lens), "p90", np.percentile(lens, 90), "max", lens.max(), "kvs", n,
      "flags", b.flags)
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
for nm, a, z in [("stage", 0, 1), ("parse + rows", 1, 2), ("look-back", 2, 3), ("meta", 3, 4),
                 ("per-row arrays", 4, 5), ("keys", 5, 6), ("values", 6, 7), ("total", 0, 7)]:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:16s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f}")
m = (st[:, 0] > 0) & (st[:, 7] > 0)
t0 = st[m, 0]
print("kernel span", t0.max() - t0.min(), "blocks stamped", int(m.sum()))
big = lens[m] > 32768
for nm, sel in (("len <= 32K", ~big), ("len > 32K", big)):
    if sel.any():
        d = (st[m, 7] - st[m, 6])[sel]
        print(f"values phase {nm}: n {int(sel.sum())} median {np.median(d):.0f} mean {np.mean(d):.0f}")
