# Transform tests and the transform bench line + trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_transforms_gpu.py tests/test_fused_seqnum_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
timeout -k 10 300 python bench.py --workload transform --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench_transform.json 2> $O/bench_transform.err || { tail -3 $O/bench_transform.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_transform.json')); print('transform', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/trace -o tf -- python3 scripts/prof_decode.py 65536 5 transform > $O/trace.log 2>&1 || exit 1
cut -d, -f1-4 $O/trace/tf_kernel_stats.csv | head -5
