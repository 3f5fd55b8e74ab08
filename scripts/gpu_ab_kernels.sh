# A/B of the row kernels on the GPU box: flat-kernel parity tests, then config-2
# bench lines for each --kernel choice.  Usage: bash scripts/gpu_ab_kernels.sh <outdir> [kernels...]
set -o pipefail
O=${1:-gpurun_out/ab_kernels}; shift
K=${@:-flat pipe}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/pytest_flat.log" 2>&1
rc=$?; tail -3 "$O/pytest_flat.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/pytest_flat.log" | head -30; exit $rc; }
for k in $K; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel $k > "$O/bench_$k.json" 2>"$O/bench_$k.err" || { tail -5 "$O/bench_$k.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$k.json')); print('$k', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
