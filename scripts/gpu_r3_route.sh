#!/bin/bash
# GEMM routing A/B for the hidden 1024 / 2048 models (same box).
set -o pipefail
O=gpurun_out/r3route
mkdir -p $O
for model in gpt-345M gpt3-1.3B; do
  for cfg in "wgrad:wgrad" "wd:wgrad,dgrad" "wdf:wgrad,dgrad,fwd" "wgrad2:wgrad"; do
    tag=${cfg%%:*}; kinds=${cfg#*:}
    FLEETX_GEMM_AUTO="$kinds" timeout -k 10 300 python bench.py --model $model --steps 20 --warmup 3 > $O/bench_${model}_$tag.log 2>&1 || { tail -20 $O/bench_${model}_$tag.log; exit 1; }
    echo "$model $tag $(grep -o '"value": [0-9.]*' $O/bench_${model}_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${model}_$tag.log) $(grep -o '"final_loss": [0-9.]*' $O/bench_${model}_$tag.log)" | tee -a $O/summary.txt
  done
done
