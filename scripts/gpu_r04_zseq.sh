# Round 4: how many sequence lanes run at once (L2 locality of the per-block
# tables): zstd text throughput and seq-kernel time per variant; a config-5
# row trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/zseq; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_physical_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
for v in base zseq48 zseq96 zseq192; do
  L=""; [ $v != base ] && L="exp/$v.so"
  PBL_LIB=$L CODEC=zstd timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/$v -o trace -- python3 scripts/prof_zstd.py 65536 3 > $O/$v.log 2>&1 || exit 1
  python3 -c "import csv; [print('$v', r['Name'][:32], round(float(r['AverageNs'])/1e3,1), 'us') for r in list(csv.DictReader(open('$O/$v/trace_kernel_stats.csv')))[:4]]"
done
timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/zipf16 -o trace -- python3 scripts/prof_decode.py 65536 5 zipf:16 > $O/zipf16.log 2>&1 || exit 1
python3 -c "import csv; [print('zipf16', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in list(csv.DictReader(open('$O/zipf16/trace_kernel_stats.csv')))[:6]]"
PBL_LIB=exp/snap_stamps.so CORPUS=words timeout -k 10 200 python scripts/snap_stamps.py 16384 > $O/snap_stamps_words.txt 2>&1 && grep -v amdgpu.ids $O/snap_stamps_words.txt
