#!/bin/bash
# Weight-gradient GEMM geometry / split-K sweep at the small-model shapes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4geom
mkdir -p $O
G=0:0,4:1,4:2,4:3,4:4,8:1,8:2,8:4
for h in 1024 1408 2048; do
  v=""; [ $h = 1024 ] && v="--vocab 50304"
  timeout -k 10 300 python tools/bench_gemm.py --hidden $h $v --only hip_wgrad_f32acc,wgrad_tn_path --gm 4 --geom $G > $O/h$h.jsonl 2>$O/h$h.err || { tail -5 $O/h$h.err; exit 1; }
done
cat $O/*.jsonl
