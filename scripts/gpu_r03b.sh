# Snappy v3 + config 5 on the flat kernel: tests and bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_physical_gpu.py tests/test_sstable_gpu.py tests/test_tables_gpu.py tests/test_baseline_configs_gpu.py tests/test_zipf_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
timeout -k 10 500 python scripts/bench_physical.py 65536 5 snappy > $O/bench_physical.json 2> $O/bench_physical.err || { tail -3 $O/bench_physical.err; exit 1; }
cat $O/bench_physical.json
for ri in 16 32; do
  timeout -k 10 300 python bench.py --workload zipf --restart-interval $ri --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/zipf_$ri.json 2> $O/zipf_$ri.err || { tail -3 $O/zipf_$ri.err; exit 1; }
  python -c "import json; d=json.load(open('$O/zipf_$ri.json')); print('zipf', $ri, d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
done
