#!/bin/bash
# Forward-overlapped AdamW footprint: isolated bandwidth of capped grids, then
# the 6.7B step under each (same box).
set -o pipefail
O=gpurun_out/r3adam
mkdir -p $O
timeout -k 10 300 python tools/bench_optim.py --capped --iters 10 > $O/bench_optim.jsonl 2>&1 || { tail -5 $O/bench_optim.jsonl; exit 1; }
cat $O/bench_optim.jsonl | grep adamw
for cfg in ${CFGS:-"128:0" "64:1" "48:1" "32:1" "96:1" "128:0"}; do
  g=${cfg%%:*}; w=${cfg#*:}
  FLEETX_ADAMW_OVERLAP_GRID=$g FLEETX_ADAMW_OVERLAP_WIDE=$w timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_${g}_${w}.log 2>&1 || { echo "FAIL $cfg"; tail -20 $O/bench_${g}_${w}.log; exit 1; }
  echo "grid=$g wide=$w $(grep -o '"value": [0-9.]*' $O/bench_${g}_${w}.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${g}_${w}.log)" | tee -a $O/summary.txt
done
