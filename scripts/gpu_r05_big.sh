# Round 5: big-block pass variants on config 5 (trace of the kernels per variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/big${TAG:-}; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
for v in ${VARIANTS}; do
  L=""; [ $v != base ] && L=exp/$v.so
  PBL_LIB=$L $B --workload zipf --restart-interval 16 > $O/${v}.json 2>$O/${v}.err || { tail -3 $O/${v}.err; exit 1; }
  python -c "import json; d=json.load(open('$O/${v}.json')); print('$v ri16', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  PBL_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o tr -- python3 scripts/prof_decode.py 65536 3 zipf:16 > $O/tr_$v.log 2>&1 || exit 1
  python -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/tr_$v/*kernel_stats.csv')[0])):
    if 'pbl' in r['Name']: print('   ', r['Name'][:60], round(float(r['AverageNs'])/1e3,1), 'us')"
done
