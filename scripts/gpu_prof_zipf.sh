set -o pipefail
mkdir -p gpurun_out/prof_zipf
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zipf -o zipf -- python3 bench.py --workload zipf --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_zipf/bench.json 2> gpurun_out/prof_zipf/err.log || { tail -20 gpurun_out/prof_zipf/err.log; exit 1; }
find gpurun_out/prof_zipf -name "*kernel_stats.csv" | head -3
for f in $(find gpurun_out/prof_zipf -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -8; done
