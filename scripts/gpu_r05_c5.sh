# Round 5: config-5 row variants (A/B on configs 5 and 2), stamps on config 5,
# row parity of the candidate.
set -o pipefail
O=gpurun_out/r05/c5${TAG:-}; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || { tail -3 $O/$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for v in ${VARIANTS:-base}; do
  L=""; [ $v != base ] && L=exp/$v.so
  PBL_LIB=$L run ${v}_ri16 --workload zipf --restart-interval 16
  PBL_LIB=$L run ${v}_ri1 --workload zipf --restart-interval 1
  PBL_LIB=$L run ${v}_ri32 --workload zipf --restart-interval 32
  PBL_LIB=$L run ${v}_cfg2
done
if [ -n "$STAMPS" ]; then WORKLOAD=zipf:16 PBL_LIB=exp/$STAMPS.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps16.txt 2>&1 && grep -v amdgpu.ids $O/stamps16.txt; fi
if [ -n "$PARITY" ]; then
  PBL_LIB=exp/$PARITY.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_row_kernels_gpu.py tests/test_zipf_gpu.py tests/test_hide_fused_gpu.py tests/test_baseline_configs_gpu.py tests/test_rowblk_gpu.py -k "not col" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
fi
