# Round-4 baseline: config-2 bench on the committed kernels (pipe / flat).
set -o pipefail
O=gpurun_out/r04/base; mkdir -p $O
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "head $git_head" > $O/head.txt
B="timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
$B > $O/bench_row.json 2>$O/bench_row.err && echo row ok && \
$B --kernel flat > $O/bench_row_flat.json 2>/dev/null && echo flat ok
