#!/usr/bin/env python3
"""Overlap of the PCIe pipeline's H2D copies (SDMA, rocprofv3 --memory-copy-trace),
D2H copies (ROCclr blit kernels __amd_rocclr_copyBuffer, --kernel-trace) and
decode kernels, inside the e2e passes of a bench run.
Usage: overlap.py <dir with m_memory_copy_trace.csv and m_kernel_trace.csv>"""
import csv
import json
import os
import sys

d = sys.argv[1]
mc = list(csv.DictReader(open(os.path.join(d, "m_memory_copy_trace.csv"))))
kt = list(csv.DictReader(open(os.path.join(d, "m_kernel_trace.csv"))))
iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))  # noqa: E731
h2d = sorted(iv(r) for r in mc if r["Direction"].endswith("HOST_TO_DEVICE"))
d2h = sorted(iv(r) for r in kt if "copyBuffer" in r["Kernel_Name"])
dec = sorted(iv(r) for r in kt if "decode_kernel" in r["Kernel_Name"] or "pipe_kernel" in r["Kernel_Name"])
# e2e window: the pipeline's decodes are the ones that overlap an H2D copy
win = [x for x in dec if any(a < x[1] and x[0] < b for a, b in h2d)]
lo, hi = (min(x[0] for x in win), max(x[1] for x in win)) if win else (0, 0)
# extend the window over the last chunk's D2H (blits starting within 5 ms of the
# last pipelined decode; the copy-engine reference copies come later)
hi = max([hi] + [x[1] for x in d2h if hi <= x[0] < hi + 5_000_000])


def clip(xs):
    return [(max(a, lo), min(b, hi)) for a, b in xs if b > lo and a < hi]


def union(xs):
    out = []
    for a, b in sorted(xs):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def inter(x, y):
    i = j = t = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        t += max(0, b - a)
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return t


H, D, K = union(clip(h2d)), union(clip(d2h)), union(clip(dec))
tot = lambda u: sum(b - a for a, b in u)  # noqa: E731
res = {"window_ms": round((hi - lo) / 1e6, 3), "h2d_busy_ms": round(tot(H) / 1e6, 3),
       "d2h_busy_ms": round(tot(D) / 1e6, 3), "decode_busy_ms": round(tot(K) / 1e6, 3),
       "h2d_and_d2h_overlap_ms": round(inter(H, D) / 1e6, 3),
       "h2d_and_decode_overlap_ms": round(inter(H, K) / 1e6, 3), "n_h2d": len(clip(h2d)), "n_d2h": len(clip(d2h)),
       "n_decode": len(clip(dec))}
print(json.dumps(res, indent=1))
