# Round 5: big-block passes (value copy with its loads issued together, the
# sizes pass in two tiers) A/B on config 5 row and config 2, then the row,
# Zipf, mixed and hide GPU tests on the in-tree build.
set -o pipefail
O=gpurun_out/r05/big2${TAG:-}; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || { tail -3 $O/$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  PBL_LIB=$L run ${v}_ri16 --workload zipf --restart-interval 16
  PBL_LIB=$L run ${v}_ri1 --workload zipf --restart-interval 1
  PBL_LIB=$L run ${v}_cfg2
done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_row_kernels_gpu.py tests/test_zipf_gpu.py tests/test_mixed_gpu.py tests/test_hide_fused_gpu.py tests/test_baseline_configs_gpu.py tests/test_fused_seqnum_gpu.py > $O/pytest.log 2>&1; tail -3 $O/pytest.log
fi
export TMPDIR=/tmp
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  rm -rf gpurun_out/prof_big2_$v
  PBL_LIB=$L timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/prof_big2_$v -o run -- python bench.py --workload zipf --restart-interval 16 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/prof_$v.log 2>&1 || exit 1
  python - $v <<'PY'
import glob,csv,sys
for f in glob.glob('gpurun_out/prof_big2_%s/**/*kernel_stats.csv' % sys.argv[1], recursive=True):
    for r in csv.DictReader(open(f)):
        if 'pbl' in r['Name']: print(sys.argv[1], r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
