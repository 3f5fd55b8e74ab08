set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== diag" && timeout -k 10 300 python scripts/zipf_diag.py 2>&1 | grep -v amdgpu.ids
echo "== diag3" && timeout -k 10 300 python scripts/zipf_diag3.py 2>&1 | grep -v amdgpu.ids
echo "== row" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline | cut -c1-140
echo "== mixed" && timeout -k 10 300 python bench.py --workload mixed --steps 5 --warmup 2 --no-cpu-baseline | cut -c1-140
