#!/bin/bash
# Round 5: persistent gemm5 for the data gradients too (with the plan's XCD-rectangle orders)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ad
mkdir -p $O
for r in 1 2; do for p in 2 1; do
  FLEETX_GEMM5_PERSIST=$p timeout -k 10 200 python3 tools/bench_gemm.py --hidden 4096 --only hip_dgrad,hip_fwd --iters 30 > $O/gemm_p${p}_$r.jsonl 2>&1 || { tail -5 $O/gemm_p${p}_$r.jsonl; exit 1; }
  echo persist=$p $r; grep gemm $O/gemm_p${p}_$r.jsonl | cut -c1-160
done; done
for r in 1 2; do for p in 2 1; do
  FLEETX_GEMM5_PERSIST=$p timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_p${p}_$r.log 2>&1 || { tail -5 $O/b67_p${p}_$r.log; exit 1; }
  echo 6.7B persist=$p $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_p${p}_$r.log)
done; done
