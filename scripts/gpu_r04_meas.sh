# Round 4: config-4 trace + PMC (the mixed path's kernels) and the physical
# bench on the current tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/meas; mkdir -p $O
PROF_BLOCKS=131072 PROF_WORKLOAD=mixed PROF_OUT=$O/mixprof bash scripts/gpu_prof.sh > $O/mixprof.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_physical.py 65536 3 snappy,zstd > $O/bench_physical.json 2> $O/bench_physical.err && cat $O/bench_physical.json
