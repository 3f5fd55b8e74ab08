"""Diagnostic: scaling of all-slow-path batches (3-byte value varints)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "zipf_diag.py")).read().split("\nrun(")[0])
for nb in (512, 2048, 8192, 32768):
    run(f"all-slow val 16K-30K nb={nb}", nb=nb, val_min=16384, val_max=30000)
for nb in (512, 8192):
    run(f"all-big val 33K-60K nb={nb}", nb=nb, val_min=33000, val_max=60000)
