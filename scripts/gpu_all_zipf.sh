# Full GPU suite, then config-5 benches.
set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for ri in 1 16 32; do
  echo "== bench zipf row ri=$ri" && timeout -k 10 300 python bench.py --workload zipf --restart-interval $ri --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_zipf_row_ri$ri.json 2> gpurun_out/bench_zipf.err || { tail -20 gpurun_out/bench_zipf.err; exit 1; }
  cut -c1-120 gpurun_out/bench_zipf_row_ri$ri.json
  grep -o '"roofline.*' gpurun_out/bench_zipf_row_ri$ri.json | cut -c1-300
done
