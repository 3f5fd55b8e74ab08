# Round 5: first GPU run of the block-resident row kernel (parity, A/B, stamps).
set -o pipefail
O=gpurun_out/r05/a; mkdir -p $O
git_head=$(cat .git_head 2>/dev/null); echo "$git_head" > $O/head.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_row_kernels_gpu.py -k res > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || { tail -5 $O/$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run pool
run res --kernel res
run pool2
PBL_LIB=exp/res_stamps.so timeout -k 10 200 python scripts/res_stamps.py > $O/stamps.txt 2>&1 && grep -v amdgpu.ids $O/stamps.txt
