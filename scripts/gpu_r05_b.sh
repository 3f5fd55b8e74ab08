# Round 5: value load/store split, keys in registers, early look-back windows:
# config-2 A/B, stamps, and row parity on the candidate build.
set -o pipefail
O=gpurun_out/r05/ab_split; mkdir -p $O
TAG=split VARIANTS="pool_valnost pool_valnold pool_nt0 pool_kr5 pool_ew4kr5 pool_ew2kr5" STAMPS=pool_ew4kr5st bash scripts/gpu_ab.sh || exit 1
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
PBL_LIB=exp/pool_ew4kr5.so $T tests/test_row_kernels_gpu.py tests/test_baseline_configs_gpu.py tests/test_hide_fused_gpu.py tests/test_zipf_gpu.py tests/test_fused_seqnum_gpu.py -k "config2 or row or hide or zipf or seq" > $O/pytest_ew4kr5.log 2>&1; tail -3 $O/pytest_ew4kr5.log
