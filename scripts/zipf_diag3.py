"""Diagnostic: slow-path cost per KV shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "zipf_diag.py")).read().split("\nrun(")[0])
run("A val 16384-16400", nb=8192, val_min=16384, val_max=16400, key_max=16)
run("B val 10000-10010", nb=8192, val_min=10000, val_max=10010, key_max=16)
run("C key 900-1024 val 100", nb=8192, key_min=900, key_max=1024, val_min=100, val_max=100)
run("D key 8-16 val 0-30000", nb=8192, key_max=16, val_max=30000)
run("E key 8-1024 val 0-100", nb=8192, val_max=100)
run("F key 300-400 val 100", nb=8192, key_min=300, key_max=400, val_min=100, val_max=100)
