# Round 4: config-2 trace + PMC of the pool kernel as built now (non-temporal
# output stores), and a zstd A/B of non-temporal write-out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/pmc2; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so; } > $O/head.txt
PROF_OUT=$O/prof bash scripts/gpu_prof.sh > $O/prof.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_physical.py 65536 3 zstd > $O/zbase.json 2>/dev/null && PBL_LIB=exp/zstd_nt.so timeout -k 10 400 python scripts/bench_physical.py 65536 3 zstd > $O/znt.json 2>/dev/null || exit 1
grep -o '"zstd[a-z_]*": {"decoded_GB_per_s": [0-9.]*' $O/zbase.json $O/znt.json
