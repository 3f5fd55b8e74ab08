set -o pipefail
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log && \
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; \
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then echo "== bench" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 3 > gpurun_out/bench.log 2>&1; tail -5 gpurun_out/bench.log; fi
