# Round 4: pool kernel with stage-holder priority — A/B over waves per CU,
# phase stamps, one SQ PMC pass.
set -o pipefail
O=gpurun_out/r04/pool2; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel pool"
for v in p16 p12 p8; do PBL_LIB=exp/pool_$v.so $B > $O/bench_$v.json 2>$O/bench_$v.err || exit 1; done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
PBL_LIB=exp/pool_p16d.so timeout -k 10 200 python scripts/pool_stamps.py > $O/pool_stamps.txt 2>&1 && cat $O/pool_stamps.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PBL_LIB=exp/pool_p16.so PROF_FLAGS=0x4000
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq1 -o sq1 -- python3 scripts/prof_decode.py 65536 3 row > $O/sq1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/sq2 -o sq2 -- python3 scripts/prof_decode.py 65536 3 row > $O/sq2.log 2>&1
echo pmc rc=$?
