# Config 5 (Zipf) on the row pipeline vs the flat kernel at restart intervals 1/16/32.
set -o pipefail
O=gpurun_out/zipf_ab; mkdir -p $O
for ri in 16 32 1; do
  for k in auto flat; do
    timeout -k 10 300 python bench.py --workload zipf --restart-interval $ri --kernel $k --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/z_${ri}_$k.json 2> $O/z_${ri}_$k.err || { tail -3 $O/z_${ri}_$k.err; exit 1; }
    python -c "import json; d=json.load(open('$O/z_${ri}_$k.json')); print('ri', $ri, '$k', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
