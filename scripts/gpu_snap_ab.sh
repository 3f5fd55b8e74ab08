# Snappy kernel A/B: physical tests on the tree, then the snappy bench on the
# tree (v3) and exp/<variant>.so.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/snap_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_physical_gpu.py tests/test_sstable_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
for v in tree "$@"; do
  if [ "$v" = tree ]; then L=""; else L="exp/$v.so"; fi
  PBL_LIB=$L timeout -k 10 500 python scripts/bench_physical.py 65536 5 ${SNAP_CODECS:-snappy} > $O/bench_$v.json 2> $O/bench_$v.err || { tail -3 $O/bench_$v.err; exit 1; }
  echo "$v $(cat $O/bench_$v.json)"
done
