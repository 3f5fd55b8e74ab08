# Round 4: pool kernel, slot re-reads instead of held registers; batch widths,
# ring vs no ring, the parker's priority kept until its stage is ready.
set -o pipefail
O=gpurun_out/r04/pool8; mkdir -p $O
cat .git_head > $O/head.txt 2>/dev/null; md5sum exp/pool_*.so >> $O/head.txt
for v in q34 q34e; do
PBL_LIB=exp/pool_$v.so timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_hide_fused_gpu.py -k 'pool or random or general or past or config2' -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; tail -1 $O/pytest_$v.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_$v.log | head -30; exit $rc; }
done
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel pool"
for v in q34 q32 q54 q34e q34p; do PBL_LIB=exp/pool_$v.so $B > $O/bench_$v.json 2>$O/bench_$v.err || exit 1; done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
for v in q34pd q34ed; do PBL_LIB=exp/pool_$v.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps_$v.txt 2>&1 && grep -v amdgpu.ids $O/stamps_$v.txt || exit 1; done
