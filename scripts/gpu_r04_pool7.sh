# Round 4: pool kernel with the first key batch / value step / restarts loaded
# before the look-back wait and software-pipelined value steps (A/B of the
# batch widths), stamps of the KU3/VG8 form.
set -o pipefail
O=gpurun_out/r04/pool7; mkdir -p $O
git rev-parse HEAD > $O/head.txt 2>/dev/null || cat .git_head > $O/head.txt 2>/dev/null
md5sum exp/pool_*.so pebble_amd/libpebble_amd.so >> $O/head.txt
PBL_LIB=exp/pool_pa.so timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_hide_fused_gpu.py -k 'pool or random or general or past or config2' -x -q --timeout 200 --timeout-method thread > $O/pytest_pa.log 2>&1; rc=$?; tail -2 $O/pytest_pa.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_pa.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel pool"
for v in pa pb pc; do PBL_LIB=exp/pool_$v.so $B > $O/bench_$v.json 2>$O/bench_$v.err || exit 1; done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
PBL_LIB=exp/pool_pad.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps_pad.txt 2>&1 && cat $O/stamps_pad.txt
