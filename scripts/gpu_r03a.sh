# Round-3 check: full GPU suite, config-2 bench line, transform bench, physical
# (snappy / zstd) bench, kernel traces for the transform and physical steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/bench_row.json 2> $O/bench_row.err || { tail -3 $O/bench_row.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_row.json')); print('row', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload transform --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench_transform.json 2> $O/bench_transform.err || { tail -3 $O/bench_transform.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_transform.json')); print('transform', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 400 python scripts/bench_physical.py 65536 5 > $O/bench_physical.json 2> $O/bench_physical.err || { tail -3 $O/bench_physical.err; exit 1; }
cat $O/bench_physical.json
R="rocprofv3 --output-format csv"
timeout -k 10 300 $R --kernel-trace --stats -d $O/tf_trace -o tf -- python3 scripts/prof_decode.py 65536 5 transform > $O/tf_trace.log 2>&1 || exit 1
timeout -k 10 300 $R --kernel-trace --stats -d $O/phys_trace -o phys -- python3 scripts/bench_physical.py 16384 3 > $O/phys_trace.log 2>&1 || exit 1
echo done
