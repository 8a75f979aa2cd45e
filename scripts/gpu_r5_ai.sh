#!/bin/bash
# Round 5: plan-driven forward routing A/B (hipBLASLt vs gemm5 where the plan
# times gemm5 >= 3 % faster) on 345M and ViT-g, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ai
mkdir -p $O
for r in 1 2; do
  for rt in off faster; do
    FLEETX_GEMM_FWD_ROUTE=$rt timeout -k 10 300 python3 bench.py --model gpt-345M --steps 30 --warmup 5 > $O/b345_${rt}_$r.log 2>&1 || { tail -5 $O/b345_${rt}_$r.log; exit 1; }
    echo "345M fwd_route=$rt run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b345_${rt}_$r.log)" | tee -a $O/summary.txt
  done
done
for r in 1 2; do
  for rt in off faster; do
    FLEETX_GEMM_FWD_ROUTE=$rt timeout -k 10 400 python3 tools/bench_vit.py --steps 10 --warmup 3 > $O/vit_${rt}_$r.log 2>&1 || { tail -5 $O/vit_${rt}_$r.log; exit 1; }
    echo "ViT-g fwd_route=$rt run $r $(tail -1 $O/vit_${rt}_$r.log)" | tee -a $O/summary.txt
  done
done
