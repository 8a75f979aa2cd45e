#!/bin/bash
# Round 5: forward routing / fused-epilogue A/B on 345M and ViT-g, interleaved:
#   off    forwards on hipBLASLt (default)
#   faster forwards on gemm5 where the plan times it >= 3 % faster
#   act    + bias+GeLU (FC1 forward) and GeLU' (FC2 data gradient) as gemm5 epilogues
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ai
mkdir -p $O
v_off="FLEETX_GEMM_FWD_ROUTE=off"
v_faster="FLEETX_GEMM_FWD_ROUTE=faster"
v_act="FLEETX_GEMM_FWD_ROUTE=off FLEETX_GEMM_AUTO=wgrad,fwd_act,dgrad_act"
v_fasteract="FLEETX_GEMM_FWD_ROUTE=faster FLEETX_GEMM_AUTO=wgrad,fwd_act,dgrad_act"
for r in 1 2; do
  for v in off faster act fasteract; do
    n=v_$v
    env ${!n} timeout -k 10 300 python3 bench.py --model gpt-345M --steps 30 --warmup 5 > $O/b345_${v}_$r.log 2>&1 || { tail -5 $O/b345_${v}_$r.log; exit 1; }
    echo "345M $v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b345_${v}_$r.log)" | tee -a $O/summary.txt
  done
done
for r in 1 2; do
  for v in off faster fasteract; do
    n=v_$v
    env ${!n} timeout -k 10 400 python3 tools/bench_vit.py --steps 10 --warmup 3 > $O/vit_${v}_$r.log 2>&1 || { tail -5 $O/vit_${v}_$r.log; exit 1; }
    echo "ViT-g $v run $r $(tail -1 $O/vit_${v}_$r.log)" | tee -a $O/summary.txt
  done
done
