# Round 4: pool-kernel wave-count variants (A/B) and the zstd plan kernel's
# wave-parallel FSE tables (physical GPU tests, physical bench, trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=waves VARIANTS="pool_w16a pool_w16b pool_w12 pool_w8rb8" bash scripts/gpu_r04_ab.sh || exit 1
TAG=d bash scripts/gpu_r04_zs.sh
