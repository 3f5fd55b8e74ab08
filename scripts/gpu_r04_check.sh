# Round 4 checkpoint on the current tree: the whole GPU suite, the smoke, the
# default bench line, then a config-2 trace + PMC of the pool kernel.
set -o pipefail
O=gpurun_out/r04/check; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so; } > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
PROF_OUT=$O/prof bash scripts/gpu_prof.sh > $O/prof.log 2>&1; tail -3 $O/prof.log
