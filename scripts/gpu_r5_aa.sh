#!/bin/bash
# Round 5: every data gradient on gemm5 (no weight transposes) vs the plan's routes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5aa
mkdir -p $O
for r in 1 2 3; do for v in wgrad wgrad,dgrad; do
  FLEETX_GEMM_AUTO=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_${v}_$r.log 2>&1 || { tail -5 $O/b67_${v}_$r.log; exit 1; }
  echo 6.7B auto=$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_${v}_$r.log)
done; done
for r in 1 2; do for v in wgrad wgrad,dgrad; do
  FLEETX_GEMM_AUTO=$v timeout -k 10 300 python3 bench.py --model gpt3-1.3B --steps 20 --warmup 5 > $O/b13_${v}_$r.log 2>&1 || { tail -5 $O/b13_${v}_$r.log; exit 1; }
  echo 1.3B auto=$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b13_${v}_$r.log)
done; done
