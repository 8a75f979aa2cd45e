#!/bin/bash
# 345M / 1.3B step A/B of the GEMM routing (same box).
set -o pipefail
O=gpurun_out/r3small
mkdir -p $O
for m in gpt-345M gpt3-1.3B; do
  for cfg in "none:" "wgrad:wgrad" "wgrad_dgrad:wgrad,dgrad"; do
    tag=${cfg%%:*}; kinds=${cfg#*:}
    FLEETX_GEMM_AUTO="$kinds" timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/bench_${m}_$tag.log 2>&1 || { echo "FAIL $m $tag"; tail -20 $O/bench_${m}_$tag.log; exit 1; }
    echo "$m $tag $(grep -o '"value": [0-9.]*' $O/bench_${m}_$tag.log) $(grep -o '"mfu": [0-9.]*' $O/bench_${m}_$tag.log)" | tee -a $O/summary.txt
  done
done
