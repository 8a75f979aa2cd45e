#!/bin/bash
# Generate the shipped GEMM plan (routes + tile orders) on an MI355X
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5plan
mkdir -p $O
timeout -k 10 900 python3 -u tools/gemm_plan.py --out $O/gemm_plan_gfx950.json > $O/plan.jsonl 2> $O/plan.err || { tail -5 $O/plan.err; exit 1; }
tail -3 $O/plan.err; wc -l $O/plan.jsonl
