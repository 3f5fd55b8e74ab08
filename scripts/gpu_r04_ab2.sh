# Round 4: depth-1 pool variants (early prefix on / off, 4 stages) against the
# default, and a kernel trace of the zstd batch path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=d1 VARIANTS="pool_noearly pool_d1 pool_d1_noearly pool_d1_s4" bash scripts/gpu_r04_ab.sh || exit 1
O=gpurun_out/r04/zstd_prof; mkdir -p $O
timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/trace -o trace -- python3 scripts/prof_zstd.py 8192 3 > $O/trace.log 2>&1 || exit 1
cat $O/trace/trace_kernel_stats.csv
