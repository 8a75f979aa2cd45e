#!/bin/bash
# Round 5: ViT-g data gradients on 128-tiles (FLEETX_GEMM5_TILE=128) vs the
# default 256-tiles (390 tiles = 1.5 waves on 256 CUs for N = 1408), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5an
mkdir -p $O
for r in 1 2; do
  for v in def t128; do
    if [ $v = t128 ]; then e="FLEETX_GEMM5_TILE=128"; else e=""; fi
    env $e timeout -k 10 400 python3 tools/bench_vit.py --steps 10 --warmup 3 > $O/vit_${v}_$r.log 2>&1 || { tail -5 $O/vit_${v}_$r.log; exit 1; }
    echo "ViT-g $v run $r $(grep -o '"value": [0-9.]*' $O/vit_${v}_$r.log | tail -1)" | tee -a $O/summary.txt
  done
done
