# A/B: working tree vs HEAD build (libpebble_amd_exp.so): GPU tests, then colblk benches (config 5 colblk, config 3).
set -o pipefail
mkdir -p gpurun_out
EXP="PBL_LIB=$PWD/pebble_amd/libpebble_amd_exp.so"
b() { timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' '; echo; }
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for i in 1 2; do
echo "== zipf col new"; b --workload zipf --zipf-format col
echo "== zipf col head"; env $EXP bash -c "$(declare -f b); b --workload zipf --zipf-format col"
done
echo "== col new"; b --workload col
echo "== col head"; env $EXP bash -c "$(declare -f b); b --workload col"
