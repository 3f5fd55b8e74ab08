# A/B of config-2 pool-kernel variants (exp/*.so, PBL_LIB) against the
# default library, plus phase stamps of $STAMPS (a PBL_STAMPS build) if set.
set -o pipefail
O=gpurun_out/r05/ab_${TAG:-x}; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so exp/*.so; } > $O/head.txt
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || exit 1; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run base
for v in $VARIANTS; do PBL_LIB=exp/$v.so run $v; done
run base2
if [ -n "$STAMPS" ]; then PBL_LIB=exp/$STAMPS.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps.txt 2>&1 && grep -v amdgpu.ids $O/stamps.txt; fi
