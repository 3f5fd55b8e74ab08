# Pipelined row kernel: row tests, stamps, bench.
set -o pipefail
mkdir -p gpurun_out
echo "== bench row (single)" && PBL_ROW_KERNEL=single timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | cut -c1-330
echo "== row gpu tests" && timeout -k 10 400 python -u -m pytest tests/test_rowblk_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_row.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_row.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_row.log; exit $rc; }
echo "== stamps" && timeout -k 10 200 python scripts/pipe_stamps.py 65536 16 2>&1 | grep -v amdgpu.ids && \
echo "== bench row (pipe)" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | cut -c1-420
