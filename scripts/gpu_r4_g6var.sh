#!/bin/bash
# VGPR-staged schedule variants (tools/gemm_lab/bin/g5v_*) vs the LDS-DMA loop, interleaved.
set -o pipefail
O=gpurun_out/r4g6var
mkdir -p $O
B=tools/gemm_lab/bin
for r in 1 2; do
  echo "== dma round $r" >> $O/var.log
  FLEETX_GEMM5_STAGE=dma timeout -k 10 120 $B/g5v_a 5 20 >> $O/var.log 2>&1 || exit 1
  for b in $B/g5v_*; do
    echo "== $(basename $b) round $r" >> $O/var.log
    timeout -k 10 120 $b 5 20 >> $O/var.log 2>&1 || exit 1
  done
done
cat $O/var.log
