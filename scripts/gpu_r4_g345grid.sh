#!/bin/bash
# 345M graph mode: deferred AdamW grid cap sweep, interleaved.
set -o pipefail
O=gpurun_out/r4g345grid
mkdir -p $O
for r in 1 2 3; do
  for g in 0 128 256 512; do
    FLEETX_ADAMW_OVERLAP_GRID=$g timeout -k 10 300 python3 bench.py --model gpt-345M --steps 40 --warmup 5 > $O/b_g${g}_$r.log 2>&1 || { tail -20 $O/b_g${g}_$r.log; exit 1; }
    echo "345M grid=$g run $r: $(tail -1 $O/b_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
  done
done
