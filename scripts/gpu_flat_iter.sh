# flat-kernel iteration on the GPU box: parity tests, A/B bench lines, phase stamps.
set -o pipefail
O=${1:-gpurun_out/flat_iter}
mkdir -p "$O"
bash scripts/gpu_ab_kernels.sh "$O" flat pipe || exit 1
timeout -k 10 300 python scripts/flat_stamps.py 65536 > "$O/stamps.txt" 2>&1; grep -v amdgpu.ids "$O/stamps.txt"
