# colblk: GPU tests, then bench col for the pipelined and the single kernel.
set -o pipefail
mkdir -p gpurun_out
echo "== col gpu tests" && timeout -k 10 400 python -u -m pytest tests/test_colblk_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_col.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_col.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_col.log; exit $rc; }
echo "== bench col (pipe)" && timeout -k 10 300 python bench.py --workload col --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | cut -c1-330 && \

echo "== stamps" && timeout -k 10 200 python scripts/col_stamps.py 65536 2>&1 | grep -v amdgpu.ids
