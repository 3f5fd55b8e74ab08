# Round 4: the pool kernel's emit reading keys from the still-held stage
# (3 / 4 stages) against the committed default; the row GPU tests on the
# 4-stage form.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=klds VARIANTS="pool_klds3 pool_klds4 pool_s4" bash scripts/gpu_r04_ab.sh || exit 1
PBL_LIB=exp/pool_klds4.so timeout -k 10 600 python -u -m pytest tests/test_row_kernels_gpu.py tests/test_rowblk_gpu.py tests/test_hide_fused_gpu.py tests/test_zipf_gpu.py tests/test_baseline_configs_gpu.py tests/test_mixed_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/ab_klds/pytest.log 2>&1; tail -2 gpurun_out/r04/ab_klds/pytest.log
