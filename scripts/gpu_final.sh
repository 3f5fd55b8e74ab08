# Round-end check of the committed tree, in two calls (each under gpurun's
# 1200 s limit):
#   PART=check  the whole GPU suite, the smoke, the default bench line (CPU
#               baseline + PCIe), bench lines for configs 1-5, the tiering,
#               hide, row-shape mix and transform workloads
#   PART=prof   a trace + PMC passes (FETCH_SIZE, WRITE_SIZE, two SQ sets)
#               per workload in PROF (default: configs 2-5), via gpu_prof.sh
# Output under gpurun_out/$R/final; scripts/summarize_prof.py copies the
# summaries into profiles/$R/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${R:-r06}
O=gpurun_out/$R/final; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so oracle/liboracle.so; } > $O/head.txt
if [ "${PART:-check}" = check ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  tail -2 $O/pytest.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log || exit 1
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
  B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
  run() { n=$1; shift; $B "$@" > $O/bench_$n.json 2>$O/bench_$n.err || exit 1; python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'])"; }
  run cfg3 --workload col; run cfg4 --workload mixed
  run cfg5_ri16 --workload zipf --restart-interval 16; run cfg5_ri32 --workload zipf --restart-interval 32
  run cfg5_ri1 --workload zipf --restart-interval 1; run cfg5_col --workload zipf --zipf-format col
  run cfg3_tier --workload col --tiering 4; run hide_row4 --hide 4; run hide_col4 --workload col --hide 4
  run rowmix_zipf10 --workload rowmix --mix zipf10; run rowmix_tail8 --workload rowmix --mix tail8
  run transform --workload transform
  timeout -k 10 200 python bench.py --workload cfg1 --no-e2e > $O/bench_cfg1.json 2> $O/bench_cfg1.err && cat $O/bench_cfg1.json || exit 1
else
  for w in ${PROF:-row col mixed zipf:16 zipf:1 zipf:32 zipf:col transform}; do
    nbp=65536; [ $w = mixed ] && nbp=131072  # (bench.py's config-4 shard)
    PROF_BLOCKS=$nbp PROF_WORKLOAD=$w PROF_OUT=$O/prof_${w/:/_} bash scripts/gpu_prof.sh > $O/prof_${w/:/_}.log 2>&1 || { tail -5 $O/prof_${w/:/_}.log; exit 1; }
    echo "prof $w done"
  done
fi
echo final done
