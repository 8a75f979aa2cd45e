#!/bin/bash
# VGPR-staged gemm5 ablations + PMC, DMA loop as the same-box baseline.
set -o pipefail
O=gpurun_out/r4g6abl
mkdir -p $O
B=tools/gemm_lab/bin
echo "== dma (g6_none, FLEETX_GEMM5_STAGE=dma)" >> $O/abl.log
FLEETX_GEMM5_STAGE=dma timeout -k 10 120 $B/g6_none 5 20 >> $O/abl.log 2>&1 || exit 1
for b in none novm nodma nowr nolds nobar; do
  echo "== g6_$b" >> $O/abl.log
  timeout -k 10 120 $B/g6_$b 5 20 >> $O/abl.log 2>&1 || exit 1
done
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE"
for st in dma vgpr; do
  FLEETX_GEMM5_STAGE=$st LAB_ONLY=out:fwd timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/pmc1_$st -o pmc -- $B/g6_none 5 5 > $O/pmc1_$st.log 2>&1 || exit 1
  FLEETX_GEMM5_STAGE=$st LAB_ONLY=out:fwd timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/pmc2_$st -o pmc -- $B/g6_none 5 5 > $O/pmc2_$st.log 2>&1 || exit 1
done
cat $O/abl.log
