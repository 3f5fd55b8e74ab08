# Traffic attribution for colblk_pipe_kernel (config 3): FETCH_SIZE / WRITE_SIZE
# of the kernel with each output component compiled out (exp/col_no*.so, built
# by scripts/build_variant.sh with -DPBL_EXP_COL_NO{ROW,KEY,VAL}) next to the
# full kernel.  Usage on the GPU box: bash scripts/col_traffic.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/coltraffic}; mkdir -p $O
P="python3 scripts/prof_decode.py 65536 3 col"
for v in full col_norow col_nokey col_noval; do
  lib=pebble_amd/libpebble_amd.so; [ $v = full ] || lib=exp/$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    PBL_LIB=$lib timeout -k 10 120 rocprofv3 --output-format csv --pmc $c -d $O/$v-$c -o x -- $P > $O/$v-$c.log 2>&1 || exit 1
  done
done
echo done
