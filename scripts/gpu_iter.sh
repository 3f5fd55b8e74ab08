set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  echo "== bench row" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids && echo "== bench col" && timeout -k 10 300 python bench.py --workload col --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids && \
  echo "== stamps" && timeout -k 10 300 python scripts/phase_stamps.py 65536 16 2>&1 | grep -v amdgpu.ids
fi
