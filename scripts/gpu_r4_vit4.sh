#!/bin/bash
# ViT-g data gradients: always gemm5 (config) vs per-shape race.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4vit4
mkdir -p $O
vit() {
  timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 $2 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
}
for r in 1 2; do
  vit cfg_$r ""
  vit race_$r "-o Engine.gemm_routing=wgrad"
done
