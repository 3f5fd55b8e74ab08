# Round 4 checkpoint: the whole GPU suite, config-2 and config-4 bench lines,
# the physical step (64 Ki distinct blocks: checksums, snappy, zstd) and a
# zstd kernel trace on the current tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/round${TAG:-}; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so; } > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
$B > $O/cfg2.json 2>$O/cfg2.err && $B --workload mixed > $O/cfg4.json 2>$O/cfg4.err || exit 1
python -c "import json; [print(n, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']) for n in ('cfg2','cfg4') for d in [json.load(open('$O/'+n+'.json'))]]"
timeout -k 10 400 python scripts/bench_physical.py 65536 3 snappy,zstd > $O/bench_physical.json 2> $O/bench_physical.err && cat $O/bench_physical.json || exit 1
timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/ztrace -o trace -- python3 scripts/prof_zstd.py 65536 3 > $O/ztrace.log 2>&1 || exit 1
cut -d, -f1-4 $O/ztrace/trace_kernel_stats.csv | head -8
