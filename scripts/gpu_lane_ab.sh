# Full GPU suite on the in-tree library, then config-2 (and config 4/5) bench
# lines of the in-tree library against exp/<variant>.so.
set -o pipefail
O=gpurun_out/lane_ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
for w in row mixed zipf; do
  for v in tree "$@"; do
    if [ "$v" = tree ]; then L=""; else L="exp/$v.so"; fi
    PBL_LIB=$L timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench_${w}_$v.json 2>$O/bench_${w}_$v.err || { tail -3 $O/bench_${w}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${w}_$v.json')); print('$w', '$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
