#!/bin/bash
# GEMM shapes of the 345M / ViT-g steps: hipBLASLt vs gemm5 (tuned tile order).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g345
mkdir -p $O
C=fwd_x_wT,fwd_x_wT_bias,dgrad_dy_w,dgrad_tn_path,wgrad_tn_path,hip_fwd,hip_fwd_bias,hip_fwd_gelu,hip_dgrad,hip_dgrad_dgelu,hip_wgrad_f32acc
timeout -k 10 300 python tools/bench_gemm.py --hidden 1024 --vocab 50304 --only $C > $O/h1024.jsonl 2>$O/h1024.err || { tail -5 $O/h1024.err; exit 1; }
timeout -k 10 300 python tools/bench_gemm.py --hidden 1536 --only $C > $O/h1536.jsonl 2>$O/h1536.err || { tail -5 $O/h1536.err; exit 1; }
timeout -k 10 300 python tools/bench_gemm.py --hidden 2048 --vocab 50304 --only $C > $O/h2048.jsonl 2>$O/h2048.err || { tail -5 $O/h2048.err; exit 1; }
cat $O/*.jsonl
