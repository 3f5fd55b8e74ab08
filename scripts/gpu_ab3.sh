# A/B: working tree (libpebble_amd.so) vs HEAD build (libpebble_amd_exp.so): row GPU tests, then row/zipf/mixed bench.
set -o pipefail
mkdir -p gpurun_out
EXP="PBL_LIB=$PWD/pebble_amd/libpebble_amd_exp.so"
b() { timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' '; echo; }
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for i in 1 2; do
echo "== row new"; b
echo "== row head"; env $EXP bash -c "$(declare -f b); b"
done
echo "== zipf new"; b --workload zipf
echo "== zipf head"; env $EXP bash -c "$(declare -f b); b --workload zipf"
echo "== mixed new"; b --workload mixed
echo "== zipf ri32 new"; b --workload zipf --restart-interval 32
echo "== zipf ri32 head"; env $EXP bash -c "$(declare -f b); b --workload zipf --restart-interval 32"
echo "== row ri32 new"; b --restart-interval 32
echo "== row ri32 head"; env $EXP bash -c "$(declare -f b); b --restart-interval 32"
