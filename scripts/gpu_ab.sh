# A/B: row GPU tests on the default kernel, then bench row for both row kernels.
set -o pipefail
mkdir -p gpurun_out
echo "== row gpu tests" && timeout -k 10 400 python -u -m pytest tests/test_rowblk_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_row.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_row.log
[ $rc -eq 0 ] || exit $rc
echo "== bench row (pipe)" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids && \
echo "== bench row (single)" && PBL_ROW_KERNEL=single timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids
