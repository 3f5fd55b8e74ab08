# Round-5 profiles of the committed build: kernel trace + PMC (FETCH_SIZE,
# WRITE_SIZE and SQ counters in separate passes) per workload, each summary
# keyed by the library's hash (scripts/summarize_prof.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/prof${TAG:-}; mkdir -p $O
for w in ${WORKLOADS:-row col zipf:16 mixed row:hide4 col:hide4}; do
  wl=${w%%:hide*}; h=0; case $w in *:hide*) h=${w##*:hide};; esac
  d=$O/$(echo $w | tr ':' '_'); nbk=65536; [ "$wl" = mixed ] && nbk=131072
  PROF_OUT=$d PROF_WORKLOAD=$wl PROF_HIDE=$h PROF_BLOCKS=$nbk bash scripts/gpu_prof.sh > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "$w ok"
done
echo prof done
