# Round 4: pool kernel variants — early stage release (metadata in the wave's
# slot, keys from global) vs the stage-held key emit; waves x stages; acquire
# back-off; unaligned 8-B LDS header reads.
set -o pipefail
O=gpurun_out/r04/pool3; mkdir -p $O
PBL_LIB=exp/pool_e10s3.so timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_hide_fused_gpu.py -k 'pool or random or general or past or config2' -x -q --timeout 200 --timeout-method thread > $O/pytest_e10s3.log 2>&1; rc=$?; tail -2 $O/pytest_e10s3.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_e10s3.log | head -30; exit $rc; }
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel pool"
for v in s8 s8ua s8w12 e10s3 e12s2 e16s2 e8s3; do PBL_LIB=exp/pool_$v.so $B > $O/bench_$v.json 2>$O/bench_$v.err || exit 1; done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in e10s3 s8; do
  PBL_LIB=exp/pool_$v.so PROF_FLAGS=0x4000 timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/ic_$v -o ic -- python3 scripts/prof_decode.py 65536 3 row > $O/ic_$v.log 2>&1 || exit 1
done
PROF_FLAGS=0x400 timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/ic_pipe -o ic -- python3 scripts/prof_decode.py 65536 3 row > $O/ic_pipe.log 2>&1
echo ic rc=$?
