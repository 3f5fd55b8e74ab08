# rocprofv3 passes for one decode workload: kernel trace + stats, FETCH_SIZE,
# WRITE_SIZE, two SQ counter sets (each pass its own run).  Env: PROF_OUT,
# PROF_BLOCKS, PROF_WORKLOAD, PROF_FLAGS (batch flags, e.g. 0x800 = flat kernel).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=${PROF_OUT:-gpurun_out/prof}; mkdir -p $D
R="rocprofv3 --output-format csv"
P="python3 scripts/prof_decode.py ${PROF_BLOCKS:-65536} 5 ${PROF_WORKLOAD:-row}"
timeout -k 10 300 $R --kernel-trace --stats -d $D/trace -o trace -- $P > $D/trace.log 2>&1 && \
timeout -s KILL 120 $R --pmc FETCH_SIZE -d $D/fetch -o fetch -- $P > $D/fetch.log 2>&1 && \
timeout -s KILL 120 $R --pmc WRITE_SIZE -d $D/write -o write -- $P > $D/write.log 2>&1 && \
timeout -s KILL 120 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/sq1 -o sq1 -- $P > $D/sq1.log 2>&1 && \
timeout -s KILL 120 $R --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d $D/sq2 -o sq2 -- $P > $D/sq2.log 2>&1 && \
timeout -s KILL 120 $R --pmc SQ_LEVEL_WAVES SQ_INSTS_SMEM SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE -d $D/sq3 -o sq3 -- $P > $D/sq3.log 2>&1
echo rc=$?
