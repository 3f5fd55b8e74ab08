# PBL_BATCH_VARLEN dispatch: GPU tests, config 5 colblk (auto = single kernel) and config 3 benches, row single-vs-pipe on config 5.
set -o pipefail
mkdir -p gpurun_out
b() { timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"kernel": "[a-z_]*"' | tr '\n' ' '; echo; }
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== zipf col auto"; b --workload zipf --zipf-format col
echo "== col"; b --workload col
echo "== zipf row pipe"; b --workload zipf
echo "== zipf row single"; PBL_ROW_KERNEL=single bash -c "$(declare -f b); b --workload zipf"
