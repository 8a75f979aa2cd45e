#!/bin/bash
# Round 6: exact packed fp32 master (26 B / parameter in the update) vs the fp32 master, 6.7B,
# 3 interleaved pairs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6v
mkdir -p $O
for r in 1 2 3; do for pm in False True; do
  FLEETX_BENCH_OVERRIDES="Optimizer.packed_master=$pm" timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_pm${pm}_$r.log 2>&1 || { tail -5 $O/b_pm${pm}_$r.log; exit 1; }
  echo packed=$pm $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_pm${pm}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b_pm${pm}_$r.log) $(grep -o '"peak_mem_gb": [0-9.]*' $O/b_pm${pm}_$r.log)
done; done
