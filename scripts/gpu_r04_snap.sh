# Round 4: snappy on the text corpus: physical GPU tests, the current kernels
# against the round-start build (exp/snap_old.so), and a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/snap${TAG:-}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_physical_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python scripts/bench_physical.py 65536 3 snappy > $O/new.json 2> $O/new.err && cat $O/new.json || exit 1
PBL_LIB=exp/snap_old.so timeout -k 10 400 python scripts/bench_physical.py 65536 3 snappy > $O/old.json 2> $O/old.err && cat $O/old.json || exit 1
CODEC=snappy timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/trace -o trace -- python3 scripts/prof_zstd.py 65536 3 > $O/trace.log 2>&1 || exit 1
python3 -c "import csv; [print(r['Name'][:44], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in list(csv.DictReader(open('$O/trace/trace_kernel_stats.csv')))[:5]]"
