# Round check: full GPU tests, smoke, bench lines (row with CPU baseline + e2e, col, mixed), rocprof trace + PMC (row, col).
set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke 2>&1 | grep -v amdgpu.ids && \
echo "== bench row" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 10 --e2e > gpurun_out/bench_row.json 2>gpurun_out/bench_row.err && cut -c1-300 gpurun_out/bench_row.json && \
echo "== bench col" && timeout -k 10 300 python bench.py --workload col --steps 10 --warmup 2 --cpu-baseline-seconds 5 > gpurun_out/bench_col.json 2>/dev/null && cut -c1-300 gpurun_out/bench_col.json && \
echo "== bench mixed" && timeout -k 10 300 python bench.py --workload mixed --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null > gpurun_out/bench_mixed.json && cut -c1-300 gpurun_out/bench_mixed.json && \
echo "== prof row" && timeout -k 10 900 bash scripts/gpu_prof.sh 2>&1 | tail -1 && mv gpurun_out/prof gpurun_out/prof_row && \
echo "== prof col" && PROF_WORKLOAD=col timeout -k 10 900 bash scripts/gpu_prof.sh 2>&1 | tail -1 && mv gpurun_out/prof gpurun_out/prof_col
