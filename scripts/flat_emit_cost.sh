# Config-2 bench lines of flat-kernel variants with parts of the emit compiled
# out (exp/<v>.so; no parity: the outputs are incomplete by construction).
# Usage: bash scripts/flat_emit_cost.sh v1 v2 ...
set -o pipefail
O=gpurun_out/flat_emit; mkdir -p $O
for v in "$@"; do
  PBL_LIB=exp/$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --kernel flat > $O/bench_$v.json 2>$O/bench_$v.err || { tail -3 $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'])"
done
