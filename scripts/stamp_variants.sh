for v in st_base st_noval st_nokey st_noarr; do echo "== $v"; PBL_LIB=exp/$v.so timeout -k 10 120 python scripts/flat_stamps.py 65536 2>&1 | grep -E "emit|total|pass|look|stage"; done
