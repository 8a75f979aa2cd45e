#!/bin/bash
# PMC counters of the attention kernels (one counter pass, no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/attn_pmc}; mkdir -p $OUT
export TMPDIR=/tmp
CTRS=${CTRS:-"GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"}
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT -o pmc -- python3 tools/bench_attention.py --iters 3 > $OUT/log.txt 2>&1
rc=$?
db=$(find $OUT -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/pmc_summary.py "$db" --filter fa_ > $OUT/summary.txt 2>&1
cat $OUT/summary.txt | head -120
exit $rc
