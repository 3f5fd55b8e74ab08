# Round 4: phase stamps of the pool kernel, early release (8 and 10 waves) vs
# keys from the stage.
set -o pipefail
O=gpurun_out/r04/pool4; mkdir -p $O
for v in e8s3d e10s3d s8d; do
  echo "== $v" && PBL_LIB=exp/pool_$v.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps_$v.txt 2>&1 && cat $O/stamps_$v.txt || exit 1
done
