#!/bin/bash
# Round 5: FC1 vs FC2 weight-gradient GEMM counters
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ah
mkdir -p $O
CTRS="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc1 -o pmc -- python3 tools/bench_wgrad_stride.py > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
db=$(find $O/pmc1 -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" --filter gemm5 > $O/pmc1_summary.txt 2>&1
CTRS2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $CTRS2 -d $O/pmc2 -o pmc -- python3 tools/bench_wgrad_stride.py > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
db=$(find $O/pmc2 -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" --filter gemm5 > $O/pmc2_summary.txt 2>&1
cat $O/pmc1_summary.txt $O/pmc2_summary.txt
