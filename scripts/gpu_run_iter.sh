# Run-major row kernel iteration: its parity tests, phase stamps (diag build),
# then A/B bench lines (run vs pipe) on config 2.
# Usage: bash scripts/gpu_run_iter.sh <outdir> [pytest -k expr]
set -o pipefail
O=${1:-gpurun_out/runk}
mkdir -p "$O"
K=${2:-"run or kernel4096"}
timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py tests/test_fused_seqnum_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|mismatch" "$O/pytest.log" | head -30; exit $rc; }
if [ -f pebble_amd/libpebble_amd_diag.so ]; then
  timeout -k 10 200 python scripts/flat_stamps.py 65536 run > "$O/stamps_run.txt" 2>&1 && grep -v amdgpu.ids "$O/stamps_run.txt" || exit 1
fi
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
$B --kernel run > "$O/bench_run.json" 2>"$O/bench_run.err" && python -c "import json;d=json.load(open('$O/bench_run.json'));print('run', d['value'], d['roofline']['kernel_ms'])" && \
$B --kernel pipe > "$O/bench_pipe.json" 2>"$O/bench_pipe.err" && python -c "import json;d=json.load(open('$O/bench_pipe.json'));print('pipe', d['value'], d['roofline']['kernel_ms'])"
