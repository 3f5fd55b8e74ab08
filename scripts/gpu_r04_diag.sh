# Round 4 diagnostics: pool-kernel phase stamps, zstd phase cycles, config-2
# A/B of pool knobs, and the read-request size mix of the pool kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/diag; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so exp/*.so; } > $O/head.txt
PBL_LIB=exp/pool_stamps.so timeout -k 10 200 python scripts/pool_stamps.py > $O/stamps.txt 2>&1 && grep -v amdgpu.ids $O/stamps.txt || exit 1
PBL_LIB=exp/zstd_prof.so timeout -k 10 300 python scripts/zstd_prof.py 8192 > $O/zstd_prof.txt 2>&1 && grep -v amdgpu.ids $O/zstd_prof.txt | tail -9 || exit 1
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/$n.json 2>$O/$n.err || exit 1; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run base; for v in vg8 ku2 prio0; do PBL_LIB=exp/pool_$v.so run $v; done
P="python3 scripts/prof_decode.py 65536 5 row"
R="rocprofv3 --output-format csv"
timeout -s KILL 120 $R --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum -d $O/rq -o rq -- $P > $O/rq.log 2>&1 || exit 1
timeout -s KILL 120 $R --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum -d $O/dram -o dram -- $P > $O/dram.log 2>&1 || exit 1
echo diag done
