#!/bin/bash
# PMC of the 345M-shape GEMMs (gemm5 data / weight gradients, hipBLASLt forward): one counter pass.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4pmc345
mkdir -p $O
CTRS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc -o pmc -- python3 tools/bench_gemm.py --tokens 8192 --hidden 1024 --iters 3 --only fwd_x_wT,hip_dgrad,hip_wgrad_f32acc > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
db=$(find $O/pmc -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" > $O/summary.txt 2>&1
head -150 $O/summary.txt
