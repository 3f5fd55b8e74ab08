# Round-3 final check: GPU tests, smoke, bench lines for configs 1-5, the
# transform and physical steps, config-5 A/B (flat vs the HBM-walking path),
# and the config-2 trace + PMC, all under gpurun_out/final3/.
set -o pipefail
O=gpurun_out/final3; mkdir -p $O
echo "== gpu tests" && timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|differs|FAIL" $O/pytest_gpu.log | head -30; exit $rc; }
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && grep smoke $O/smoke.log || exit 1
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2"
$B --cpu-baseline-seconds 10 > $O/bench_row.json 2>$O/bench_row.err && echo row ok && \
$B --workload col --cpu-baseline-seconds 5 > $O/bench_col.json 2>/dev/null && echo col ok && \
$B --workload mixed --no-cpu-baseline > $O/bench_mixed.json 2>/dev/null && echo mixed ok && \
$B --workload transform --no-cpu-baseline --no-e2e > $O/bench_transform.json 2>/dev/null && echo transform ok && \
$B --workload zipf --restart-interval 1 --no-cpu-baseline > $O/bench_zipf_ri1.json 2>/dev/null && \
$B --workload zipf --restart-interval 16 --cpu-baseline-seconds 5 > $O/bench_zipf_ri16.json 2>/dev/null && \
$B --workload zipf --restart-interval 32 --no-cpu-baseline > $O/bench_zipf_ri32.json 2>/dev/null && \
$B --workload zipf --zipf-format col --no-cpu-baseline > $O/bench_zipf_col.json 2>/dev/null && echo zipf ok && \
timeout -k 10 300 python bench.py --workload cfg1 > $O/bench_cfg1.json 2>/dev/null && echo cfg1 ok && \
timeout -k 10 400 python scripts/bench_physical.py > $O/bench_physical.json 2>/dev/null && echo physical ok || exit 1
G="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --workload zipf --kernel global"
for ri in 16 32 1; do $G --restart-interval $ri > $O/ab_zipf_global_$ri.json 2>/dev/null || exit 1; done; echo global ab ok
PROF_OUT=$O/prof timeout -k 10 900 bash scripts/gpu_prof.sh > $O/prof.log 2>&1 && echo prof ok
