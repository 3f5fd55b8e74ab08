# GPU check of the working tree: the GPU suite (or TESTS), the smoke, and
# bench lines for the workloads in BENCH (default: configs 2 and 3).
#   TAG=name TESTS="tests/test_x.py" BENCH="row col mixed" bash scripts/gpu_check.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-check}; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so oracle/liboracle.so; } > $O/head.txt
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}
  timeout -k 10 1000 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
fi
if [ -n "${SMOKE:-}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log || exit 1
fi
B="timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/bench_$n.json 2>$O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', round(d['value'],1), d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline'].get('traffic'))"; }
for w in ${BENCH:-row col}; do
  case $w in
    row) run row ;;
    col) run col --workload col ;;
    mixed) run mixed --workload mixed ;;
    zipf16) run zipf16 --workload zipf --restart-interval 16 ;;
    zipf32) run zipf32 --workload zipf --restart-interval 32 ;;
    zipf1) run zipf1 --workload zipf --restart-interval 1 ;;
    zipfcol) run zipfcol --workload zipf --zipf-format col ;;
    coltier) run coltier --workload col --tiering 4 ;;
    hiderow) run hiderow --hide 4 ;;
    hidecol) run hidecol --workload col --hide 4 ;;
    transform) run transform --workload transform ;;
    none) ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
done
echo check done
