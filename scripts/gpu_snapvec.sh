# Development run: full GPU suite on the in-tree library, then the
# PBL_SNAPPY_VEC=1 variant (exp/snapvec.so) on the physical-step tests and bench.
set -o pipefail
O=gpurun_out/snapvec; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_physical.py > $O/bench_physical_head.json 2>/dev/null && cat $O/bench_physical_head.json || exit 1
PBL_LIB=exp/snapvec.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "physical or snappy or sstable" > $O/pytest_snapvec.log 2>&1
rc=$?; tail -n 2 $O/pytest_snapvec.log; [ $rc -eq 0 ] || exit $rc
PBL_LIB=exp/snapvec.so timeout -k 10 400 python scripts/bench_physical.py > $O/bench_physical_snapvec.json 2>/dev/null && cat $O/bench_physical_snapvec.json
