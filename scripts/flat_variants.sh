# A/B of flat-kernel variants (exp/<v>.so): parity tests of the first, stamps
# (exp/st_<v>.so when present) and config-2 bench lines of each.
# Usage: bash scripts/flat_variants.sh v1 v2 ...
set -o pipefail
O=gpurun_out/flat_variants; mkdir -p $O
PBL_LIB=exp/$1.so timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head; exit 1; }
for v in "$@"; do
  if [ -f exp/st_$v.so ]; then echo "== stamps $v"; PBL_LIB=exp/st_$v.so timeout -k 10 120 python scripts/flat_stamps.py 65536 2>&1 | grep -E "emit|total|pass|look|stage"; fi
  PBL_LIB=exp/$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel flat > $O/bench_$v.json 2>$O/bench_$v.err || { tail -3 $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'])"
done
