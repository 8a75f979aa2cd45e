#!/bin/bash
# Round 5: forward GEMMs (and GeLU epilogues) on gemm5 in the 6.7B step, after XCD rectangles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
for r in 1 2; do for v in wgrad wgrad,fwd wgrad,fwd,fwd_act wgrad,fwd,fwd_act,dgrad_act; do
  FLEETX_GEMM_AUTO=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_${v}_$r.log 2>&1 || { tail -5 $O/b67_${v}_$r.log; exit 1; }
  echo 6.7B auto=$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_${v}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b67_${v}_$r.log)
done; done
