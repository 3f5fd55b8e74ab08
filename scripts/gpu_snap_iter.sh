# Snappy iteration: physical tests, stamps (exp/snapst.so), snappy bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/snap_iter; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_physical_gpu.py tests/test_sstable_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
PBL_LIB=exp/snapst.so timeout -k 10 300 python scripts/snap_stamps.py 16384 2>&1 | grep -v amdgpu.ids | tee $O/stamps.txt
timeout -k 10 500 python scripts/bench_physical.py 65536 5 snappy > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
cat $O/bench.json
