#!/bin/bash
# gemm5 tile-order M-group (gm) sweep on the 6.7B shapes vs hipBLASLt, one process per round.
set -o pipefail
O=gpurun_out/${OUT:-r4gm}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_gemm.py --iters 30 --gm 1,2,4,8,16 \
    --only fwd_x_wT,dgrad_tn_path,hip_fwd,hip_dgrad,hip_wgrad_f32acc >> $O/gm.jsonl 2>> $O/gm.err || exit 1
done
grep -v amdgpu $O/gm.jsonl
