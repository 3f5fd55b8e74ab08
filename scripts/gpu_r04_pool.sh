# Round 4: staging-pool row kernel parity (pool params of the row-kernel
# suite) + MinLZ device tests, then config-2 bench A/B (pipe, pool, pool-w12).
set -o pipefail
O=gpurun_out/r04/pool; mkdir -p $O
echo "head $(cat .git_head 2>/dev/null)" > $O/head.txt
timeout -k 10 400 python -u -m pytest tests/test_flat_gpu.py tests/test_fused_seqnum_gpu.py tests/test_physical_gpu.py -k "pool or 16384 or minlz" -x -q --timeout 200 --timeout-method thread > $O/pytest_pool.log 2>&1; rc=$?; tail -3 $O/pytest_pool.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_pool.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
$B --kernel pipe > $O/bench_pipe.json 2>$O/bench_pipe.err && echo pipe ok && \
$B --kernel pool > $O/bench_pool.json 2>$O/bench_pool.err && echo pool ok && \
PBL_LIB=exp/pool_w12.so $B --kernel pool > $O/bench_pool_w12.json 2>$O/bench_pool_w12.err && echo w12 ok
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
[ -f exp/pool_diag.so ] && PBL_LIB=exp/pool_diag.so timeout -k 10 200 python scripts/pool_stamps.py > $O/pool_stamps.txt 2>&1 && cat $O/pool_stamps.txt
