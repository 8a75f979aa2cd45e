#!/bin/bash
# Decode: GEMV cold vs Infinity-Cache-warm weights, generation baseline.
set -o pipefail
O=gpurun_out/r3dec
mkdir -p $O
timeout -k 10 300 python tools/bench_gemv.py --m 1 4 --warm > $O/gemv_warm.jsonl 2>&1 || { tail -5 $O/gemv_warm.jsonl; exit 1; }
grep shape $O/gemv_warm.jsonl
timeout -k 10 300 python tools/bench_generation.py --model gpt3-1.3B --batch 1 4 --fused-only > $O/gen_1.3B.jsonl 2>&1 || { tail -5 $O/gen_1.3B.jsonl; exit 1; }
grep ms_per_token $O/gen_1.3B.jsonl
