# Round-final check: GPU tests, smoke, bench lines for configs 1, 2 (CPU baseline + e2e), 3, 4 shard,
# 5 (RI 1/16/32, colblk) and the physical step, saved under gpurun_out/final/.
set -o pipefail
mkdir -p gpurun_out/final
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/final/pytest_gpu.log; exit $rc; }
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/final/smoke.log 2>&1 && cat gpurun_out/final/smoke.log | grep smoke
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2"
$B --cpu-baseline-seconds 10 > gpurun_out/final/bench_row.json 2>gpurun_out/final/bench_row.err && echo row ok && \
$B --workload col --cpu-baseline-seconds 5 > gpurun_out/final/bench_col.json 2>/dev/null && echo col ok && \
$B --workload mixed --no-cpu-baseline > gpurun_out/final/bench_mixed.json 2>/dev/null && echo mixed ok && \
$B --workload zipf --restart-interval 1 --no-cpu-baseline > gpurun_out/final/bench_zipf_ri1.json 2>/dev/null && \
$B --workload zipf --restart-interval 16 --cpu-baseline-seconds 5 > gpurun_out/final/bench_zipf_ri16.json 2>/dev/null && \
$B --workload zipf --restart-interval 32 --no-cpu-baseline > gpurun_out/final/bench_zipf_ri32.json 2>/dev/null && \
$B --workload zipf --zipf-format col --no-cpu-baseline > gpurun_out/final/bench_zipf_col.json 2>/dev/null && echo zipf ok && \
timeout -k 10 300 python bench.py --workload cfg1 > gpurun_out/final/bench_cfg1.json 2>/dev/null && echo cfg1 ok && \
timeout -k 10 400 python scripts/bench_physical.py > gpurun_out/final/bench_physical.json 2>/dev/null && echo physical ok
echo "== trace zipf col" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/trace_zipf_col -o t -- python3 bench.py --workload zipf --zipf-format col --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/final/trace_zipf_col.log 2>&1 && \
find gpurun_out/final/trace_zipf_col -name "*kernel_stats.csv" | head -1
