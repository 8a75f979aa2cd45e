#!/bin/bash
# Interleaved A/B of gemm5 schedule variants (tools/gemm_lab/bin/g5v_*), ROUNDS rounds.
set -o pipefail
O=gpurun_out/g5var
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for b in tools/gemm_lab/bin/g5v_*; do
    echo "== $(basename $b) round $r" >> $O/var.log
    timeout -k 10 120 $b 5 20 >> $O/var.log 2>&1 || exit 1
  done
done
