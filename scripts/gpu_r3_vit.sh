#!/bin/bash
# ViT-g/14 GEMM routing A/B on one box: weight gradients only (default) vs
# + data gradients / forward / fused-GeLU epilogues on the MFMA kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3vit
mkdir -p $O
for a in wgrad wgrad,dgrad wgrad,fwd wgrad,dgrad_act wgrad,fwd_act wgrad; do
  FLEETX_GEMM_AUTO=$a timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/bench_$a.log 2>&1 || { tail -20 $O/bench_$a.log; exit 1; }
  echo "auto=$a $(tail -1 $O/bench_$a.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
done
