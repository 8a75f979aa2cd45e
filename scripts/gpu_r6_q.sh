#!/bin/bash
# Round 6: FC1 fused forward on gemm5 with and without the forward-overlapped AdamW
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6q
mkdir -p $O
for r in 1 2; do for ov in True False; do for v in wgrad wgrad,fwd_act; do
  FLEETX_BENCH_OVERRIDES="Distributed.comm.overlap_optimizer=$ov" FLEETX_GEMM_AUTO=$v timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_${ov}_${v}_$r.log 2>&1 || { tail -5 $O/b_${ov}_${v}_$r.log; exit 1; }
  echo overlap=$ov auto=$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${ov}_${v}_$r.log)
done; done; done
