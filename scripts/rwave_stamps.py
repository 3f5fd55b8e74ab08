#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of the two-pass row emit kernel
(rowblk_wave.hip.h, PBL_STAMPS build) on config 5's row batch.
Stamps: 0 start, 1 bases read + block metadata written, 2 staged,
3 LDS walk done (the metadata pass on the lane-parallel form), 5 keys and
per-KV arrays written (lane-parallel form, wave 0), 6 values written (wave 1
of a two-wave workgroup), 7 long keys' own bytes and restarts (wave 2 of a
three-wave workgroup), 4 end (wave 0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PBL_LIB", os.path.join(ROOT, "pebble_amd", "libpebble_amd_diag.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.batch import BlockBatch, decode, decode_into, gen_zipf_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ri = int(sys.argv[2]) if len(sys.argv) > 2 else 16
if len(sys.argv) > 3 and sys.argv[3] == "row":  # config 2's blocks, the two-pass form forced
    from pebble_amd.rowblk import gen_row_blocks
    buf, off, lens, n = gen_row_blocks(42, nb, 32768, ri, 16, 100, n_threads=16)
else:
    buf, off, lens, n = gen_zipf_blocks(42, nb, N.PBL_FMT_ROW, ri, 32768, n_threads=16)
b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, N.PBL_BATCH_VARLEN)
print("blocks: len median", np.median(lens), "p90", np.percentile(lens, 90), "max", lens.max(), "kvs", n,
      "flags", hex(b.flags))
for _ in range(3):
    out = decode(b)
torch.cuda.synchronize()
# one more launch with the stamp words cleared, timed by HIP events (the
# s_memtime clock against wall time)
ws_stamps = 256 + 10 * nb * 8
out.workspace[ws_stamps: ws_stamps + nb * 16 * 8].zero_()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
decode_into(b, out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
ws_state = 256 + 10 * nb * 8
st = out.workspace[ws_state: ws_state + nb * 16 * 8].view(torch.int64).view(nb, 16).cpu().numpy()
nkv = np.diff(out.blk_kv_base.cpu().numpy())[:nb]
for nm, a, z in [("bases + meta", 0, 1), ("stage (DMA)", 1, 2), ("LDS walk", 2, 3), ("global walk", 3, 4), ("keys (wave 0)", 3, 5), ("values (wave 1)", 3, 6), ("long keys (wave 2)", 3, 7),
                 ("total", 0, 4)]:
    m = (st[:, a] > 0) & (st[:, z] > 0)
    d = (st[m, z] - st[m, a]).astype(np.float64)
    if d.size:
        print(f"{nm:14s} median {np.median(d):9.0f} mean {np.mean(d):9.0f} p90 {np.percentile(d, 90):9.0f}")
m = (st[:, 2] > 0) & (st[:, 3] > 0)
d = (st[m, 3] - st[m, 2]).astype(np.float64)
k = nkv[m].astype(np.float64)
print("LDS walk per entry: median", np.median(d / np.maximum(k, 1)), "KVs per block mean", k.mean())
print(f"whole decode {ms:.3f} ms (size + scan + emit)")
