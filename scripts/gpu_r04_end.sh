# Round 4 end: the whole GPU suite, the smoke, the default bench line and the
# config 3 / 4 lines on the committed tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/end; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so oracle/liboracle.so; } > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
$B --workload col > $O/bench_cfg3.json 2>/dev/null && $B --workload mixed > $O/bench_cfg4.json 2>/dev/null || exit 1
python -c "import json; [print(n, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic']) for n in ('bench_cfg3','bench_cfg4') for d in [json.load(open('$O/'+n+'.json'))]]"
