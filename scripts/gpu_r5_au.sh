#!/bin/bash
# Round 5: shipped vendor GEMM tuning off / on for GPT-3 1.3B, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5au
mkdir -p $O
for r in 1 2; do
  for v in off on; do
    FLEETX_VENDOR_TUNE=$v timeout -k 10 400 python3 bench.py --model gpt3-1.3B --steps 20 --warmup 5 > $O/b13_${v}_$r.log 2>&1 || { tail -5 $O/b13_${v}_$r.log; exit 1; }
    echo "gpt3-1.3B vendor_tune=$v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b13_${v}_$r.log)" | tee -a $O/summary.txt
  done
done
