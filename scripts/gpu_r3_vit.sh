#!/bin/bash
# ViT-g/14 GEMM routing A/B on one box: weight gradients only (default) vs
# + data gradients vs + forward on the MFMA kernel (128 x 128 tiles for the
# 1408-wide shapes), then a kernel trace of the winner.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3vit
mkdir -p $O
for a in wgrad wgrad,dgrad wgrad,dgrad,fwd wgrad,fwd; do
  FLEETX_GEMM_AUTO=$a timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/bench_$a.log 2>&1 || { tail -20 $O/bench_$a.log; exit 1; }
  echo "auto=$a $(tail -1 $O/bench_$a.log)" | tee -a $O/summary.txt
done
