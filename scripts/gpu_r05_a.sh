# Round 5: first GPU run of the block-resident row kernel (parity, A/B, stamps)
# plus the tests of this round's other changes.
set -o pipefail
O=gpurun_out/r05/a; mkdir -p $O
cat .git_head > $O/head.txt 2>/dev/null
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
$T tests/test_row_kernels_gpu.py -k res > $O/pytest_res.log 2>&1 || { tail -40 $O/pytest_res.log; exit 1; }
tail -2 $O/pytest_res.log
$T tests/test_hide_fused_gpu.py tests/test_mixed_gpu.py tests/test_physical_gpu.py tests/test_zipf_gpu.py tests/test_fused_seqnum_gpu.py tests/test_baseline_configs_gpu.py -k "minlz or mixed or hide or zipf_row or row_batches or ab_flags or config2" > $O/pytest_other.log 2>&1 || { tail -40 $O/pytest_other.log; exit 1; }
tail -2 $O/pytest_other.log
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || { tail -5 $O/$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run pool
run res --kernel res
run pool2
PBL_LIB=exp/res_stamps.so timeout -k 10 200 python scripts/res_stamps.py > $O/stamps.txt 2>&1 && grep -v amdgpu.ids $O/stamps.txt
