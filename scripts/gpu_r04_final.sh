# Round 4 final check on the committed tree: the whole GPU suite, the smoke,
# the default bench line (CPU baseline + PCIe), bench lines for configs 1-5,
# the row-shape mixes and the transform pass, a config-2 trace + PMC of the
# pool kernel, and PMC of the zstd batch path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/final${TAG:-}; mkdir -p $O
{ cat .git_head 2>/dev/null; md5sum pebble_amd/libpebble_amd.so oracle/liboracle.so; } > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest.log | head -40; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() { n=$1; shift; $B "$@" > $O/bench_$n.json 2>$O/bench_$n.err || exit 1; python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'])"; }
run cfg3 --workload col; run cfg4 --workload mixed
run cfg5_ri16 --workload zipf --restart-interval 16; run cfg5_ri32 --workload zipf --restart-interval 32
run cfg5_ri1 --workload zipf --restart-interval 1; run cfg5_col --workload zipf --zipf-format col
run rowmix_zipf10 --workload rowmix --mix zipf10; run rowmix_tail8 --workload rowmix --mix tail8
run transform --workload transform
timeout -k 10 200 python bench.py --workload cfg1 --no-e2e > $O/bench_cfg1.json 2> $O/bench_cfg1.err && cat $O/bench_cfg1.json || exit 1
PROF_OUT=$O/prof bash scripts/gpu_prof.sh > $O/prof.log 2>&1 || exit 1
R="rocprofv3 --output-format csv"
P="python3 scripts/prof_zstd.py 65536 3"
timeout -s KILL 200 $R --pmc FETCH_SIZE -d $O/zfetch -o fetch -- $P > $O/zfetch.log 2>&1 || exit 1
timeout -s KILL 200 $R --pmc WRITE_SIZE -d $O/zwrite -o write -- $P > $O/zwrite.log 2>&1 || exit 1
timeout -s KILL 200 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/zsq -o sq -- $P > $O/zsq.log 2>&1 || exit 1
echo final done
