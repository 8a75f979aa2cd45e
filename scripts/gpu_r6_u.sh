#!/bin/bash
# Round 6: uncapped head units of the overlapped update (root + layer 0 gate the first
# forward kernels), 6.7B, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6u
mkdir -p $O
for r in 1 2 3; do for h in 0 2; do
  FLEETX_ADAMW_HEAD=$h timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_h${h}_$r.log 2>&1 || { tail -5 $O/b_h${h}_$r.log; exit 1; }
  echo head=$h $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_h${h}_$r.log)
done; done
