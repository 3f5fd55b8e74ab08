# Config-5 (zipf, row RI 16) rocprofv3 trace + PMC passes, then the config-5 bench lines for RI 1/16/32.
set -o pipefail
mkdir -p gpurun_out
PROF_WORKLOAD=zipf timeout -k 10 900 bash scripts/gpu_prof.sh > gpurun_out/prof_zipf.log 2>&1; rc=$?; tail -3 gpurun_out/prof_zipf.log
[ $rc -eq 0 ] || exit $rc
for ri in 1 16 32; do
  timeout -k 10 300 python bench.py --workload zipf --restart-interval $ri --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_zipf_ri$ri.json 2>/dev/null || exit 1
  cut -c1-160 gpurun_out/bench_zipf_ri$ri.json
done
