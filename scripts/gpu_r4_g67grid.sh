#!/bin/bash
# 6.7B whole-step graph: deferred AdamW grid uncapped (default) vs 128 / 256 workgroups, interleaved.
set -o pipefail
O=gpurun_out/r4g67grid
mkdir -p $O
for r in 1 2; do
  for g in 0 128 256; do
    FLEETX_ADAMW_OVERLAP_GRID=$g timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/b_g${g}_$r.log 2>&1 || { tail -20 $O/b_g${g}_$r.log; exit 1; }
    echo "grid=$g run $r: $(tail -1 $O/b_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' | tr '\n' ' ')" | tee -a $O/summary.txt
  done
done
