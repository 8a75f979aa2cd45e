#!/bin/bash
# Round 4: VGPR-staged gemm5 K-loop -- numerics, then an A/B against the
# LDS-DMA loop and hipBLASLt on the 6.7B layer shapes (same box).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1
rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_gemm.py --iters 20 --stages 0,1 \
    --only fwd_x_wT,dgrad_tn_path,wgrad_tn_path,hip_fwd,hip_dgrad,hip_wgrad_f32acc,hip_fwd_gelu,hip_dgrad_dgelu >> $O/bench_gemm.jsonl 2>> $O/bench_gemm.err || exit 1
done
grep -v amdgpu $O/bench_gemm.jsonl
