# Full GPU check: tests, smoke, bench lines for each workload (+ e2e for row).
set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -6 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke 2>&1 | grep -v amdgpu.ids && \
echo "== bench row" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 5 --e2e 2>&1 | grep -v amdgpu.ids && \
echo "== bench col" && timeout -k 10 300 python bench.py --workload col --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids && \
echo "== bench mixed" && timeout -k 10 300 python bench.py --workload mixed --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids
echo "== bench zipf" && timeout -k 10 300 python bench.py --workload zipf --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | cut -c1-400
