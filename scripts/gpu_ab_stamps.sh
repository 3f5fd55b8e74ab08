# Development run: row-pipeline phase stamps + role placement (diag build), A/B of
# exp/*.so against the in-tree library on config 2, and the row GPU parity tests.
# Usage (on the GPU box via gpurun): bash scripts/gpu_ab_stamps.sh <outdir> [pytest -k expr]
set -o pipefail
O=${1:-gpurun_out/abst}
mkdir -p "$O"
K=${2:-row}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -n 3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
if [ -f pebble_amd/libpebble_amd_diag.so ]; then
  timeout -k 10 200 python scripts/pipe_stamps.py 65536 16 > "$O/stamps.txt" 2>&1 || exit 1
  cat "$O/stamps.txt"
fi
bash scripts/ab.sh "$O/ab"
for w in $AB_WORKLOADS; do bash scripts/ab.sh "$O/ab_$w" --workload $w || exit 1; done
