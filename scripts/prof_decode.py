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
hide = int(os.environ.get("PROF_HIDE", "0"))  # bench.py --hide N: every N-th KV obsolete, hidden
if workload == "col":
    from pebble_amd import _native as N
    from pebble_amd.colblk import gen_col_blocks
    buf, off, lens, n = gen_col_blocks(42, nb, 32768, n_threads=16, obsolete_every=hide)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_COL_CRDB1, N.PBL_ROW_HIDE_OBSOLETE if hide else 0)
elif workload.startswith("zipf"):
    # config 5 (bench.py --workload zipf): "zipf" / "zipf:RI" row format at
    # restart interval RI (default 16), "zipf:col" colblk DefaultKeySchema
    from pebble_amd import _native as N
    from pebble_amd.batch import gen_zipf_blocks
    arg = workload.split(":")[1] if ":" in workload else "16"
    fmt = N.PBL_FMT_COL_DEFAULT if arg == "col" else N.PBL_FMT_ROW
    ri = 16 if arg == "col" else int(arg)
    buf, off, lens, n = gen_zipf_blocks(42, nb, fmt, ri, 32768, n_threads=16)
    b = BlockBatch.from_host(buf, off, lens, "cuda", fmt, 0)
elif workload == "mixed":
    # config 4 shard: even ids row (config-2 shape), odd ids colblk crdb1 (config-3 shape)
    import numpy as np
    from pebble_amd import _native as N
    from pebble_amd.colblk import gen_col_blocks
    h = nb // 2
    rb, ro, rl, rn = gen_row_blocks(42, nb - h, 32768, 16, 16, 100, n_threads=16)
    cb, co, cl, cn = gen_col_blocks(42, h, 32768, n_threads=16)
    buf = np.zeros(nb * 32768 + 16, np.uint8)
    v = buf[: nb * 32768].reshape(nb, 32768)
    v[0::2] = rb[: (nb - h) * 32768].reshape(nb - h, 32768)
    v[1::2] = cb[: h * 32768].reshape(h, 32768)
    off = np.arange(nb, dtype=np.uint64) * 32768
    lens = np.empty(nb, np.uint32)
    lens[0::2], lens[1::2] = rl, cl
    bf = np.empty(nb, np.uint8)
    bf[0::2], bf[1::2] = N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1
    n = rn + cn
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, 0, block_format=bf)
else:
    from pebble_amd import _native as N
    buf, off, lens, n = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16, obsolete_every=hide)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, N.PBL_ROW_HIDE_OBSOLETE if hide else 0)
b.flags |= int(os.environ.get("PROF_FLAGS", "0"), 0)  # e.g. PBL_KERNEL_PIPE (0x400) for A/B profiles
if workload == "transform":
    # the config-2 batch decoded once, then transformed `iters` times
    from pebble_amd.transforms import TransformPlan, Transforms
    d = decode(b)
    plan = TransformPlan(d, Transforms(synthetic_seq_num=12345, hide_obsolete_points=True,
                                       synthetic_prefix=b"tenant-0042/"))
    for _ in range(iters):
        plan.launch()
    torch.cuda.synchronize()
    print("ok", n)
    sys.exit(0)
h = decode(b).to_host()
out = DecodedBatch.allocate(nb, Capacity(h["n_kv"], h["key_bytes_total"], h["val_bytes_total"], h["n_restarts"]),
                            "cuda")
for _ in range(iters):
    decode_into(b, out)
torch.cuda.synchronize()
print("ok", n)
