# A/B: working tree (libpebble_amd.so) vs HEAD build (libpebble_amd_exp.so), same box.
set -o pipefail
mkdir -p gpurun_out
EXP="PBL_LIB=$PWD/pebble_amd/libpebble_amd_exp.so"
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for i in 1 2; do
echo "== row new" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' '; echo
echo "== row head" && env $EXP timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' '; echo
done
echo "== col new" && timeout -k 10 300 python bench.py --workload col --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*' ; echo
echo "== col head" && env $EXP timeout -k 10 300 python bench.py --workload col --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*'; echo
echo "== zipf new" && timeout -k 10 300 python bench.py --workload zipf --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*'; echo
