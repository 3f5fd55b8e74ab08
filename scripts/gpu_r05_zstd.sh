# Round 5: zstd batch-path variants: GPU tests of the physical step on the
# variant, then the physical bench (zstd) and a kernel trace of the text corpus.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/zstd${TAG:-}; mkdir -p $O
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  if [ $v != base ]; then
    PBL_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_physical_gpu.py > $O/pytest_$v.log 2>&1; rc=$?; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest_$v.log | head; exit 1; }
  fi
  PBL_LIB=$L timeout -k 10 400 python scripts/bench_physical.py 65536 5 ${CODECS:-zstd} > $O/phys_$v.json 2> $O/phys_$v.err || { tail -3 $O/phys_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/phys_$v.json')); print('$v', {k: (v['decoded_GB_per_s'], v['ratio']) for k, v in d.items() if isinstance(v, dict) and 'ratio' in v})"
  PBL_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o tr -- python3 scripts/prof_zstd.py 65536 3 > $O/tr_$v.log 2>&1 || exit 1
  python -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/tr_$v/*kernel_stats.csv')[0])):
    if 'zstd' in r['Name']: print('   ', r['Name'][:50], round(float(r['AverageNs'])/1e6,3), 'ms')"
done
