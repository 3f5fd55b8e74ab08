"""Diagnostic: decode time of config-5 variants (which blocks are slow?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pebble_amd import _native as N
from pebble_amd.batch import BlockBatch, Capacity, DecodedBatch, decode, decode_into, gen_zipf_blocks


def run(name, **kw):
    buf, off, lens, n = gen_zipf_blocks(42, kw.pop("nb", 65536), N.PBL_FMT_ROW, **kw)
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, 0)
    h = decode(b).to_host()
    cap = Capacity(kv=h["n_kv"], key=h["key_bytes_total"], val=h["val_bytes_total"], rst=h["n_restarts"])
    out = DecodedBatch.allocate(len(off), cap, "cuda")
    s = torch.cuda.current_stream()
    decode_into(b, out, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(3):
        decode_into(b, out, s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    ib = int(lens.astype(np.int64).sum())
    print(f"{name:40s} blocks={len(off)} big={(lens > 32768).sum()} kvs/blk={n / len(off):.1f} "
          f"mean_len={lens.mean():.0f} slow={h['n_slow_blocks']} ms={ms:.3f} GiB/s={ib / ms / 1e-3 / 2**30:.1f}",
          flush=True)


run("zipf ri16")
run("zipf ri16 val<=8K", val_max=8192)
run("zipf ri16 val<=30K", val_max=30000)
run("zipf ri16 key<=64", key_max=64)
run("zipf ri16 key<=64 val<=1K", key_max=64, val_max=1024)
run("zipf ri16 8192 blocks", nb=8192)
os.environ["PBL_ROW_KERNEL"] = "single"
run("single: zipf ri16")
run("single: zipf ri16 val<=8K", val_max=8192)
