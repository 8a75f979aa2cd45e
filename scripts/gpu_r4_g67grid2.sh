#!/bin/bash
# Graph-mode deferred AdamW grid: 6.7B at 64 / 128 / 192, 1.3B uncapped vs 128, interleaved.
set -o pipefail
O=gpurun_out/r4g67grid2
mkdir -p $O
for r in 1 2; do
  for g in 64 128 192; do
    FLEETX_ADAMW_OVERLAP_GRID=$g timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/b67_g${g}_$r.log 2>&1 || { tail -20 $O/b67_g${g}_$r.log; exit 1; }
    echo "6.7B grid=$g run $r: $(tail -1 $O/b67_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
  done
  for g in 0 128; do
    FLEETX_ADAMW_OVERLAP_GRID=$g timeout -k 10 300 python bench.py --model gpt3-1.3B --steps 20 --warmup 3 > $O/b13_g${g}_$r.log 2>&1 || { tail -20 $O/b13_g${g}_$r.log; exit 1; }
    echo "1.3B grid=$g run $r: $(tail -1 $O/b13_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
  done
done
