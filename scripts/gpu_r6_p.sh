#!/bin/bash
# Round 6: 6.7B step with the FC1 forward (bias+GeLU epilogue) and/or the FC2 data gradient
# (GeLU' epilogue) on gemm5, vs the default routes; interleaved, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6p
mkdir -p $O
for r in 1 2; do for v in wgrad wgrad,fwd_act wgrad,fwd_act,dgrad_act; do
  FLEETX_GEMM_AUTO=$v timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b67_${v}_$r.log 2>&1 || { tail -5 $O/b67_${v}_$r.log; exit 1; }
  echo 6.7B auto=$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_${v}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b67_${v}_$r.log)
done; done
