#!/bin/bash
# Round 5: AdamW overlap grid cap sweep on the 6.7B default step (bf16 gradients)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5x
mkdir -p $O
for r in 1 2; do for g in 128 96 160 192; do
  FLEETX_BENCH_OVERRIDES="Distributed.comm.overlap_optimizer_grid=$g" timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_g${g}_$r.log 2>&1 || { tail -5 $O/b67_g${g}_$r.log; exit 1; }
  echo 6.7B grid=$g $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_g${g}_$r.log)
done; done
