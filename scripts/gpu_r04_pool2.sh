# Round 4: pool kernel with stage-holder priority — A/B over waves per CU,
# config 5 and row-shape mixes on pool vs the current routing, phase stamps,
# SQ PMC passes.
set -o pipefail
O=gpurun_out/r04/pool2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_hide_fused_gpu.py -k 'pool or hide or fused or random or general or past or config2 or colblk' -x -q --timeout 200 --timeout-method thread > $O/pytest_p16.log 2>&1; rc=$?; tail -2 $O/pytest_p16.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_p16.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
for v in p16 p16v1 p12; do PBL_LIB=exp/pool_$v.so $B --kernel pool > $O/bench_$v.json 2>$O/bench_$v.err || exit 1; done
for ri in 16 32 1; do PBL_LIB=exp/pool_p16.so $B --kernel pool --workload zipf --restart-interval $ri > $O/bench_zipf_pool_$ri.json 2>$O/err_z$ri || exit 1; done
for m in zipf10 tail8; do
  $B --workload rowmix --mix $m > $O/bench_mix_auto_$m.json 2>$O/err_ma$m || exit 1
  PBL_LIB=exp/pool_p16.so $B --workload rowmix --mix $m --kernel pool > $O/bench_mix_pool_$m.json 2>$O/err_mp$m || exit 1
done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
PBL_LIB=exp/pool_p16d.so timeout -k 10 200 python scripts/pool_stamps.py > $O/pool_stamps.txt 2>&1 && cat $O/pool_stamps.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PBL_LIB=exp/pool_p16.so PROF_FLAGS=0x4000
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq1 -o sq1 -- python3 scripts/prof_decode.py 65536 3 row > $O/sq1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/sq2 -o sq2 -- python3 scripts/prof_decode.py 65536 3 row > $O/sq2.log 2>&1
echo pmc rc=$?
