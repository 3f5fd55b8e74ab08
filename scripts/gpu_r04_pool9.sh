# Round 4: compact slots and two blocks in flight per wave (default build),
# against one block per wave; batch widths; stamps.
set -o pipefail
O=gpurun_out/r04/pool9; mkdir -p $O
cat .git_head > $O/head.txt 2>/dev/null; md5sum pebble_amd/libpebble_amd.so exp/pool_*.so >> $O/head.txt
timeout -k 10 600 python -u -m pytest tests/test_row_kernels_gpu.py tests/test_hide_fused_gpu.py tests/test_rowblk_gpu.py tests/test_fused_seqnum_gpu.py tests/test_zipf_gpu.py tests/test_baseline_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || exit 1; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run cfg2; run cfg2_pipe --kernel pipe
for v in d1 d2k4 d2v8; do PBL_LIB=exp/pool_$v.so run cfg2_$v; done
run mix_tail8 --workload rowmix --mix tail8; run mix_zipf10 --workload rowmix --mix zipf10; run z16 --workload zipf --restart-interval 16
PBL_LIB=exp/pool_d2s.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps_d2s.txt 2>&1 && grep -v amdgpu.ids $O/stamps_d2s.txt
PBL_LIB=exp/zstd_prof.so timeout -k 10 300 python scripts/zstd_prof.py 8192 > $O/zstd_prof.txt 2>&1; grep -v amdgpu.ids $O/zstd_prof.txt | tail -9
