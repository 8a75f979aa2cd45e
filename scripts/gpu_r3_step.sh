#!/bin/bash
# 6.7B step A/B of the GEMM routing (same box): FLEETX_GEMM_AUTO sets.
set -o pipefail
O=gpurun_out/r3step
mkdir -p $O
for cfg in "none:" "default:wgrad,dgrad,dgrad_act,fwd_act" "all:wgrad,dgrad,dgrad_act,fwd_act,fwd" "wgrad:wgrad"; do
  tag=${cfg%%:*}; kinds=${cfg#*:}
  FLEETX_GEMM_AUTO="$kinds" timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/bench_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $O/bench_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.log) $(grep -o '"final_loss": [0-9.]*' $O/bench_$tag.log)" | tee -a $O/summary.txt
done
