#!/bin/bash
# 6.7B graph mode: deferred AdamW cap around 128 (112 / 128 / 144 / 160), interleaved.
set -o pipefail
O=gpurun_out/r4g67grid3
mkdir -p $O
for r in 1 2; do
  for g in 112 128 144 160; do
    FLEETX_ADAMW_OVERLAP_GRID=$g timeout -k 10 400 python3 bench.py --steps 10 --warmup 4 > $O/b_g${g}_$r.log 2>&1 || { tail -20 $O/b_g${g}_$r.log; exit 1; }
    echo "6.7B grid=$g run $r: $(tail -1 $O/b_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
  done
done
