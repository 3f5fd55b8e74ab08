# Round 5: value-pipeline depth A/B on config 2, stamps and row parity of the
# candidate (exp/pool_k1v8d2.so).
set -o pipefail
O=gpurun_out/r05/ab_vd2; mkdir -p $O
TAG=vd2 VARIANTS="pool_k1v8d2 pool_k1v8d2w4 pool_k1v6d2 pool_k1v10d2" STAMPS=pool_k1v8d2st bash scripts/gpu_ab.sh || exit 1
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
PBL_LIB=exp/pool_k1v8d2.so $T tests/test_row_kernels_gpu.py tests/test_baseline_configs_gpu.py tests/test_hide_fused_gpu.py tests/test_zipf_gpu.py tests/test_fused_seqnum_gpu.py tests/test_mixed_gpu.py -k "config2 or row or hide or zipf or seq or mixed" > $O/pytest_k1v8d2.log 2>&1; tail -3 $O/pytest_k1v8d2.log
