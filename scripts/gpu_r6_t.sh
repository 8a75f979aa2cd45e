#!/bin/bash
# Round 6: one-pass LayerNorm backward + column sums at h 4096 (FLEETX_LN_BWD_FUSED=2) vs
# the row kernel + column-tile passes, 6.7B step, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_norm_gpu.py > $O/t.log 2>&1 || { echo FAIL; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do for m in 1 2; do
  FLEETX_LN_BWD_FUSED=$m timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_m${m}_$r.log 2>&1 || { tail -5 $O/b_m${m}_$r.log; exit 1; }
  echo fused=$m $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_m${m}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b_m${m}_$r.log)
done; done
