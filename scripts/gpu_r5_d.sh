#!/bin/bash
# Round 5: persistent gemm5 with the next tile's DMA prologue under the epilogue
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_gemm.log 2>&1 || { tail -30 $O/test_gemm.log; exit 1; }
tail -2 $O/test_gemm.log
for h in 4096 1024; do
for p in 1 0; do
FLEETX_GEMM5_PERSIST=$p timeout -k 10 300 python3 -u tools/bench_gemm.py --hidden $h --only fwd_x_wT,hip_fwd,hip_fwd_bias,hip_fwd_gelu,dgrad_tn_path,hip_dgrad,hip_dgrad_dgelu --iters 30 > $O/gemm_h${h}_p$p.jsonl 2> $O/gemm_h${h}_p$p.err || { tail -5 $O/gemm_h${h}_p$p.err; exit 1; }
echo "h=$h persist=$p"; cat $O/gemm_h${h}_p$p.jsonl
done
done
