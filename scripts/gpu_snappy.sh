# Physical-step tests and the physical bench (snappy / zstd).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/snap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_physical_gpu.py tests/test_sstable_gpu.py tests/test_tables_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
timeout -k 10 500 python scripts/bench_physical.py 65536 5 ${SNAP_CODECS:-snappy} > $O/bench_physical.json 2> $O/bench_physical.err || { tail -3 $O/bench_physical.err; exit 1; }
cat $O/bench_physical.json
