# Round 4: snappy4's dependency passes: the physical GPU tests, the physical
# bench (64 Ki distinct blocks, snappy), and the text-corpus phase stamps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/snap2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_physical_gpu.py tests/test_tables_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python scripts/bench_physical.py 65536 3 snappy > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
PBL_LIB=exp/snap_stamps.so CORPUS=words timeout -k 10 200 python scripts/snap_stamps.py 16384 > $O/stamps.txt 2>&1 && grep -v amdgpu.ids $O/stamps.txt
