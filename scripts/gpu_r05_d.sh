# Round 5: unified key+value steps A/B on config 2, stamps, row parity of uni1.
set -o pipefail
O=gpurun_out/r05/ab_uni; mkdir -p $O
TAG=uni VARIANTS="pool_k1v8d2 pool_uni1 pool_uni2" STAMPS=pool_uni1st bash scripts/gpu_ab.sh || exit 1
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
PBL_LIB=exp/pool_uni1.so $T tests/test_row_kernels_gpu.py tests/test_baseline_configs_gpu.py tests/test_hide_fused_gpu.py tests/test_zipf_gpu.py tests/test_fused_seqnum_gpu.py tests/test_mixed_gpu.py -k "config2 or row or hide or zipf or seq or mixed" > $O/pytest_uni1.log 2>&1; tail -3 $O/pytest_uni1.log
