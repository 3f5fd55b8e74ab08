# A/B of library variants on the default bench workload (no CPU baseline).
# Usage: bash scripts/ab.sh <outdir> <bench args...>; variants = exp/*.so plus the in-tree build.
set -o pipefail
O=${1:-gpurun_out/ab}; shift
mkdir -p "$O"
run() {  # name lib bench-args...
  local n=$1 lib=$2; shift 2
  PBL_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e "$@" > "$O/$n.json" 2>"$O/$n.err" || return 1
  python -c "import json,sys; d=json.load(open('$O/$n.json')); print('%-12s %8.1f GiB/s  kernel %.4f ms  frac %.4f' % ('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
}
for rep in 1 2; do
  run head$rep pebble_amd/libpebble_amd.so "$@" || exit 1
  for f in exp/*.so; do n=$(basename $f .so); run $n$rep $f "$@" || exit 1; done
done
