# Round 5: config 5 (row RI 16/1/32, colblk) variants after the in-kernel
# big-block walk; colblk Zipf on the pipeline against the one-block kernel.
set -o pipefail
O=gpurun_out/r05/c5b${TAG:-}; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || { tail -3 $O/$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  PBL_LIB=$L run ${v}_ri16 --workload zipf --restart-interval 16
  PBL_LIB=$L run ${v}_ri1 --workload zipf --restart-interval 1
  PBL_LIB=$L run ${v}_ri32 --workload zipf --restart-interval 32
  [ -n "$CFG2" ] && PBL_LIB=$L run ${v}_cfg2
done
if [ -n "$COL" ]; then
  run col_single --workload zipf --zipf-format col
  run col_pipe --workload zipf --zipf-format col --kernel pipe
fi
