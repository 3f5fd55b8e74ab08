# Round 4, last check: snappy4's dependency passes (physical tests, bench,
# stamps), then the whole GPU suite, the smoke and the default bench line on
# the same tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r04_snap2.sh || exit 1
O=gpurun_out/r04/last; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so oracle/liboracle.so; } > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json
