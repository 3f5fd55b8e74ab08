set -o pipefail
run() { echo "$1 $(env $2 timeout -k 10 300 python bench.py $3 --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ')"; }
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for i in 1 2; do
run new "X=1" ""
run head "PBL_LIB=$PWD/pebble_amd/libpebble_amd_exp.so" ""
done
run zipf "X=1" "--workload zipf"
