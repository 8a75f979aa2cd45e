#!/bin/bash
# gemm5 lab on one GPU: ablation timings (tools/gemm_lab/build_g5_abl.sh) and
# two PMC passes of the unablated kernel on LAB_ONLY cases.
set -o pipefail
O=gpurun_out/g5lab
mkdir -p $O
B=tools/gemm_lab/bin
for b in ${BINS:-g5_none g5_novm g5_nodma g5_nobar g5_nolds g5_nodma_nolds}; do
  echo "== $b" >> $O/abl.log
  timeout -k 10 120 $B/$b 5 20 >> $O/abl.log 2>&1 || exit 1
done
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE"
for c in ${PMC_CASES:-fc1:fwd out:fwd fc2:dgrad}; do
  t=${c//:/_}
  LAB_ONLY=$c timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/pmc1_$t -o pmc -- $B/g5_none 5 5 > $O/pmc1_$t.log 2>&1 || exit 1
  LAB_ONLY=$c timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/pmc2_$t -o pmc -- $B/g5_none 5 5 > $O/pmc2_$t.log 2>&1 || exit 1
done
