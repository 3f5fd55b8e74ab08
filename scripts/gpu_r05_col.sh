# Round 5: colblk pipeline variants (A/B on config 3 and its fused hide), then
# the colblk GPU tests on the first variant.
set -o pipefail
O=gpurun_out/r05/col${TAG:-}; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || { tail -3 $O/$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  PBL_LIB=$L run ${v}_cfg3 --workload col
  PBL_LIB=$L run ${v}_hide --workload col --hide 4
done
if [ -n "$PARITY" ]; then
  PBL_LIB=exp/$PARITY.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_colblk_gpu.py tests/test_hide_fused_gpu.py tests/test_mixed_gpu.py tests/test_baseline_configs_gpu.py tests/test_zipf_gpu.py > $O/pytest.log 2>&1; tail -3 $O/pytest.log
fi
if [ -n "$MIXED" ]; then
  for v in ${VARIANTS}; do L=""; [ $v != base ] && L=exp/$v.so; PBL_LIB=$L run ${v}_cfg4 --workload mixed; PBL_LIB=$L run ${v}_cfg5col --workload zipf --zipf-format col; done
fi
