#!/bin/bash
# 6.7B / 1.3B: whole-step HIP graph (deferred overlapped AdamW) vs eager, interleaved.
set -o pipefail
O=gpurun_out/r4g67
mkdir -p $O
for r in 1 2; do
  for g in 0 1; do
    timeout -k 10 400 python bench.py --steps 10 --warmup 3 --hip-graph $g > $O/b67_g${g}_$r.log 2>&1 || { tail -20 $O/b67_g${g}_$r.log; exit 1; }
    echo "6.7B graph=$g run $r: $(tail -1 $O/b67_g${g}_$r.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
  done
done
for g in 0 1; do
  timeout -k 10 300 python bench.py --model gpt3-1.3B --steps 10 --warmup 3 --hip-graph $g > $O/b13_g$g.log 2>&1 || { tail -20 $O/b13_g$g.log; exit 1; }
  echo "1.3B graph=$g: $(tail -1 $O/b13_g$g.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/summary.txt
done
