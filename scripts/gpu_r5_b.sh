#!/bin/bash
# Round 5 probe 2: the update split into per-unit launches (as in the step)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py --chunks 66 --only qkv,fc1 > $O/beside66.jsonl 2> $O/beside66.err || { tail -5 $O/beside66.err; exit 1; }
cat $O/beside66.jsonl
timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py --chunks 8 --only qkv,fc1 > $O/beside8.jsonl 2> $O/beside8.err || { tail -5 $O/beside8.err; exit 1; }
cat $O/beside8.jsonl
