# Round 4: the physical GPU tests, the physical bench (64 Ki distinct blocks),
# and kernel traces of zstd and snappy on the text corpus.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/zs${TAG:-}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_physical_gpu.py tests/test_tables_gpu.py tests/test_sstable_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python scripts/bench_physical.py 65536 3 snappy,zstd > $O/bench_physical.json 2> $O/bench_physical.err && cat $O/bench_physical.json || exit 1
for c in zstd snappy; do
  CODEC=$c timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/$c -o trace -- python3 scripts/prof_zstd.py 65536 3 > $O/$c.log 2>&1 || exit 1
  python3 -c "import csv; [print(r['Name'][:44], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in list(csv.DictReader(open('$O/$c/trace_kernel_stats.csv')))[:6]]"
done
