#!/usr/bin/env python3
"""Summarize a scripts/gpu_prof.sh run (gpurun_out/prof) into profiles/<tag>_*.

Writes <tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats output, copied),
<tag>_pmc.json (per-dispatch means of every counter for the decode kernel) and
profiles/pmc_traffic.json (HBM bytes per launch, gfx950-corrected per
MI355X_MICROARCH.md §HBM: FETCH_SIZE x 2 for 16-B/lane streaming reads,
WRITE_SIZE as is; both in KiB).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.environ.get("PROF_SRC", os.path.join(ROOT, "gpurun_out", "prof"))
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "rowblk_pipe_kernel"
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
WORKLOAD = sys.argv[4] if len(sys.argv) > 4 else "row"
HIDE = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # bench.py --hide N / PROF_HIDE=N
LIB_SHA = open(os.path.join(src, "lib_sha.txt")).read().strip() if os.path.exists(os.path.join(src, "lib_sha.txt")) else None

shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
pmc = collections.defaultdict(list)
# KERNEL may name several kernels joined by "+" (a decode made of several
# launches, e.g. the mixed path): per-dispatch means and trace averages are
# summed over them
KERNELS = KERNEL.split("+")
for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        for k in KERNELS:
            if k + "(" in r["Kernel_Name"] or k + "<" in r["Kernel_Name"]:
                pmc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
means = collections.defaultdict(float)
for (k, c), v in pmc.items():
    means[c] += sum(v) / len(v)
means = dict(means)
stats = {}
for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv"))):
    for k in KERNELS:
        if k + "(" in r["Name"] or k + "<" in r["Name"]:
            if not stats:
                stats = {"calls": int(r["Calls"]), "avg_ns": 0.0, "min_ns": 0.0, "max_ns": 0.0}
            stats["avg_ns"] += float(r["AverageNs"])
            stats["min_ns"] += float(r["MinNs"])
            stats["max_ns"] += float(r["MaxNs"])
out = {"kernel": KERNEL, "workload_blocks": NB, "lib_sha16": LIB_SHA, "hide": HIDE, "trace": stats,
       "pmc_per_dispatch_mean": means}
if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
    fetch = means["FETCH_SIZE"] * 2 * 1024
    write = means["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = fetch + write
    base = ("pmc_traffic" if WORKLOAD == "row" else "pmc_traffic_zipf" if WORKLOAD == "zipf:col" else
            f"pmc_traffic_{WORKLOAD.replace(':', '_ri')}")
    tname = base + (f"_hide{HIDE}" if HIDE else "") + ".json"
    json.dump({"kernel": KERNEL, "workload": WORKLOAD.split(":")[0], "workload_blocks": NB, "block_size": 32768,
               "lib_sha16": LIB_SHA, "hide": HIDE,
               "fetch_bytes_corrected": fetch, "write_bytes": write,
               **(({"restart_interval": 16, "zipf_format": "col"} if WORKLOAD == "zipf:col" else
                   {"restart_interval": int(WORKLOAD.split(":")[1]) if ":" in WORKLOAD else 16, "zipf_format": "row"})
                  if WORKLOAD.startswith("zipf") else {}),
               "hbm_bytes_per_launch": fetch + write,
               "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; FETCH_SIZE(KiB)x2x1024 "
                         "(gfx950 16-B/lane streaming-read correction), WRITE_SIZE(KiB)x1024",
               "source": f"profiles/{tag}_pmc.json"}, open(os.path.join(dst, tname), "w"), indent=1)
json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
