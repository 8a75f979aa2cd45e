#!/bin/bash
# Forward-GEMM race A/B (FLEETX_GEMM_ROUTE_KINDS=dgrad,fwd) on 6.7B and ViT-g, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4fwd
mkdir -p $O
run() {  # tag, env, args
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("gemm_raced_to_kernel"))')" | tee -a $O/summary.txt
}
vit() {
  env $2 timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
}
for r in 1 2 3; do
  run fwd_$r "FLEETX_GEMM_ROUTE_KINDS=dgrad,fwd" "--steps 10 --warmup 3"
  run dgrad_$r "FLEETX_GEMM_ROUTE_KINDS=dgrad" "--steps 10 --warmup 3"
done
for r in 1 2; do
  vit vit_fwd_$r "FLEETX_GEMM_ROUTE_KINDS=dgrad,fwd"
  vit vit_dgrad_$r "FLEETX_GEMM_ROUTE_KINDS=dgrad"
done
