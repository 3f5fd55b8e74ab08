# Round 4: pool kernel, early stage release with batched global loads in the
# key and value emits (8 waves x 3 stages), parity + bench + stamps.
set -o pipefail
O=gpurun_out/r04/pool5; mkdir -p $O
PBL_LIB=exp/pool_ee8.so timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_hide_fused_gpu.py -k 'pool or random or general or past or config2' -x -q --timeout 200 --timeout-method thread > $O/pytest_ee8.log 2>&1; rc=$?; tail -2 $O/pytest_ee8.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_ee8.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel pool"
for v in ee8 ee8vg4 n12; do PBL_LIB=exp/pool_$v.so $B > $O/bench_$v.json 2>$O/bench_$v.err || exit 1; done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
PBL_LIB=exp/pool_ee8d.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps_ee8d.txt 2>&1 && cat $O/stamps_ee8d.txt
