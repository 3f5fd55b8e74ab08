# Round 5: snappy variants: GPU tests of the physical step on the variant,
# the physical bench (snappy, both corpora) and phase stamps on the text corpus.
set -o pipefail
O=gpurun_out/r05/snap${TAG:-}; mkdir -p $O
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  if [ $v != base ]; then
    PBL_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_physical_gpu.py > $O/pytest_$v.log 2>&1; rc=$?; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest_$v.log | head; exit 1; }
  fi
  PBL_LIB=$L timeout -k 10 400 python scripts/bench_physical.py 65536 5 snappy > $O/phys_$v.json 2> $O/phys_$v.err || { tail -3 $O/phys_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/phys_$v.json')); print('$v', {k: (v['decoded_GB_per_s'], v['ratio']) for k, v in d.items() if isinstance(v, dict) and 'ratio' in v})"
done
for st in ${STAMPS}; do
  CORPUS=words PBL_LIB=exp/$st.so timeout -k 10 200 python scripts/snap_stamps.py 16384 > $O/stamps_$st.txt 2>&1 && echo "== $st" && grep -v amdgpu.ids $O/stamps_$st.txt
done
