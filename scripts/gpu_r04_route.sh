# Round 4: the pool kernel (default build) against the current routes on every
# row workload: config 2, the row-shape mixes, config 5 at RI 1 / 16 / 32.
set -o pipefail
O=gpurun_out/r04/route; mkdir -p $O
cat .git_head > $O/head.txt 2>/dev/null; md5sum pebble_amd/libpebble_amd.so >> $O/head.txt
timeout -k 10 400 python -u -m pytest tests/test_flat_gpu.py tests/test_hide_fused_gpu.py tests/test_fused_seqnum_gpu.py tests/test_zipf_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || exit 1; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run cfg2_auto; run cfg2_pool --kernel pool
for m in zipf10 tail8; do run mix_${m}_auto --workload rowmix --mix $m; run mix_${m}_pool --workload rowmix --mix $m --kernel pool; done
for ri in 1 16 32; do run z${ri}_auto --workload zipf --restart-interval $ri; run z${ri}_pool --workload zipf --restart-interval $ri --kernel pool; done
