#!/usr/bin/env python3
"""Diagnostic: the two-pass row form (rowblk_wave.hip.h) forced onto a batch
with PBL_BATCH_VARLEN, against the staging-pool kernel, on config 2 (fixed
32 KiB blocks) or config 5; run under rocprofv3 --kernel-trace --stats for the
per-kernel split.  usage: row_wave_probe.py [row|zipf] [n_blocks]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.batch import BlockBatch, decode, decode_into  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "row"
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
if wl == "row":
    from pebble_amd.rowblk import gen_row_blocks
    buf, off, lens, n = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
else:
    from pebble_amd.batch import gen_zipf_blocks
    buf, off, lens, n = gen_zipf_blocks(42, nb, N.PBL_FMT_ROW, 16, 32768, n_threads=16)
for name, fl in (("wave", N.PBL_BATCH_VARLEN), ("pool", N.PBL_KERNEL_POOL)):
    b = BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, fl)
    out = decode(b)
    h = out.to_host()
    assert h["n_kv"] == n and h["status_mask"] == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    decode_into(b, out)
    ev[0].record()
    for _ in range(5):
        decode_into(b, out)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 5
    print(f"{wl} {name}: {ms:.3f} ms/decode, {b.input_bytes() / ms / 1e6 / 1.073741824:.1f} GiB/s")
