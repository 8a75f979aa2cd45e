#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=tools/gemm_lab/bin
for gm in 2 4 8 16 32; do
  echo "GM=$gm"
  FLEETX_GEMM_GM=$gm timeout -k 10 120 $B/gemm_lab_abl0 0 10 || exit 1
done 2>&1 | tee gpurun_out/lab2.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc2 -o pmc -- $B/gemm_lab_abl0 0 5 > gpurun_out/pmc2.log 2>&1
echo "pmc rc=$?"
