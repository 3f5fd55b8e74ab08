# Config 5 (Zipf) parity tests and bench lines.
set -o pipefail
mkdir -p gpurun_out
echo "== zipf gpu tests" && timeout -k 10 400 python -u -m pytest tests/test_zipf_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_zipf.log 2>&1; rc=$?; tail -12 gpurun_out/pytest_zipf.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_zipf.log; exit $rc; }
for ri in 1 16 32; do
  echo "== bench zipf row ri=$ri" && timeout -k 10 300 python bench.py --workload zipf --restart-interval $ri --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_zipf_row_ri$ri.json 2> gpurun_out/bench_zipf.err || { tail -20 gpurun_out/bench_zipf.err; exit 1; }
  cut -c1-700 gpurun_out/bench_zipf_row_ri$ri.json
done
echo "== bench zipf col" && timeout -k 10 300 python bench.py --workload zipf --zipf-format col --steps 10 --warmup 2 > gpurun_out/bench_zipf_col.json 2> gpurun_out/bench_zipf.err || { tail -20 gpurun_out/bench_zipf.err; exit 1; }
cut -c1-900 gpurun_out/bench_zipf_col.json
