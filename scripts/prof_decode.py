#!/usr/bin/env python3
"""Profiling driver: decode one config-2 (row) or config-3 (col) batch `iters` times (for rocprofv3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pebble_amd.batch import BlockBatch, Capacity, DecodedBatch, decode, decode_into  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
workload = sys.argv[3] if len(sys.argv) > 3 else "row"
if workload == "col":
    from pebble_amd import _native as N
    from pebble_amd.colblk import gen_col_blocks
    buf, off, lens, n = gen_col_blocks(42, nb, 32768, n_threads=16)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_CRDB1, 0)
elif workload == "zipf":
    # config 5, row format, restart interval 16 (bench.py --workload zipf)
    from pebble_amd import _native as N
    from pebble_amd.batch import gen_zipf_blocks
    buf, off, lens, n = gen_zipf_blocks(42, nb, N.PBL_FMT_ROW, 16, 32768, n_threads=16)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, 0)
else:
    buf, off, lens, n = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
    b = BlockBatch.from_host(buf, off, lens, "cuda")
h = decode(b).to_host()
out = DecodedBatch.allocate(nb, Capacity(h["n_kv"], h["key_bytes_total"], h["val_bytes_total"], h["n_restarts"]),
                            "cuda")
for _ in range(iters):
    decode_into(b, out)
torch.cuda.synchronize()
print("ok", n)
