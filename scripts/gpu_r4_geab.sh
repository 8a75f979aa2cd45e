#!/bin/bash
# Same-box A/B of the shipped default (graph, 128-cap deferred update) vs eager, driver command, interleaved.
set -o pipefail
O=gpurun_out/r4geab
mkdir -p $O
for r in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --hip-graph $g > $O/b_g${g}_$r.log 2>&1 || { tail -20 $O/b_g${g}_$r.log; exit 1; }
    echo "graph=$g run $r: $(tail -1 $O/b_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
  done
done
