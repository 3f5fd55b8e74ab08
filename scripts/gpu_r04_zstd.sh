# Round 4: the zstd batch path (zstd_fast.hip.h): the physical GPU tests, then
# zstd throughput against the one-wave-per-block path (exp/zstd_old.so).
set -o pipefail
O=gpurun_out/r04/zstd; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so exp/*.so; } > $O/head.txt
timeout -k 10 300 python -u -m pytest tests/test_physical_gpu.py tests/test_tables_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/bench_physical.py 16384 3 zstd > $O/bench_new.json 2> $O/bench_new.err && cat $O/bench_new.json || exit 1
PBL_LIB=exp/zstd_old.so timeout -k 10 300 python scripts/bench_physical.py 16384 2 zstd > $O/bench_old.json 2> $O/bench_old.err && cat $O/bench_old.json
