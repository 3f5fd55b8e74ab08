set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=${PROF_OUT:-gpurun_out/prof}; mkdir -p $D
# the library the profiled process loads (PBL_LIB or the in-tree build): the
# summary records its hash, and bench.py quotes a traffic file only for it
python3 -c "import hashlib,os; p=os.environ.get('PBL_LIB') or 'pebble_amd/libpebble_amd.so'; print(hashlib.sha256(open(p,'rb').read()).hexdigest()[:16])" > $D/lib_sha.txt
R="rocprofv3 --output-format csv"
P="python3 scripts/prof_decode.py ${PROF_BLOCKS:-65536} 5 ${PROF_WORKLOAD:-row}"
timeout -k 10 300 rocprofv3 -L > $D/counters_list.txt 2>&1; \
timeout -k 10 300 $R --kernel-trace --stats -d $D/trace -o trace -- $P > $D/trace.log 2>&1 && \
timeout -k 10 300 $R --pmc FETCH_SIZE -d $D/fetch -o fetch -- $P > $D/fetch.log 2>&1 && \
timeout -k 10 300 $R --pmc WRITE_SIZE -d $D/write -o write -- $P > $D/write.log 2>&1 && \
timeout -k 10 300 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/sq1 -o sq1 -- $P > $D/sq1.log 2>&1 && \
timeout -k 10 300 $R --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d $D/sq2 -o sq2 -- $P > $D/sq2.log 2>&1
echo rc=$?
find $D -name "*.csv" | head -30
