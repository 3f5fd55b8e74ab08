set -o pipefail
mkdir -p gpurun_out
echo "== stamps" && timeout -k 10 300 python scripts/phase_stamps.py 65536 16 2>&1 | grep -v amdgpu.ids && \
echo "== prof" && timeout -k 10 900 bash scripts/gpu_prof.sh 2>&1 | tail -3
