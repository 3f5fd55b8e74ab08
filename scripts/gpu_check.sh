# GPU check used during development: GPU tests, smoke, default bench line.
# Usage (on the GPU box via gpurun): bash scripts/gpu_check.sh <outdir> [pytest -k expr]
set -o pipefail
O=${1:-gpurun_out/check}
mkdir -p "$O"
K=${2:+-k "$2"}
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread $K > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/pytest_gpu.log" | head -30; exit $rc; }
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 && grep smoke "$O/smoke.log" && \
echo "== bench" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 8 > "$O/bench_row.json" 2>"$O/bench_row.err" && cat "$O/bench_row.json"
