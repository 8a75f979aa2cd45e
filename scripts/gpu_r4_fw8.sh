#!/bin/bash
# Forward workgroup width A/B (4 vs 8 waves) at the GPT shapes.
set -o pipefail
O=gpurun_out/r4fw8
mkdir -p $O
for w in 4 8 4 8; do
  FLEETX_FA_FWD_WAVES=$w timeout -k 10 200 python -u tools/bench_attention.py --iters 40 >> $O/d128_w$w.jsonl 2>&1 || exit 1
  FLEETX_FA_FWD_WAVES=$w timeout -k 10 200 python -u tools/bench_attention.py --iters 40 --h 16 --d 64 >> $O/d64_w$w.jsonl 2>&1 || exit 1
done
for f in $O/*.jsonl; do echo "== $f"; grep -o '"causal": [a-z]*, "dropout": [0-9.]*, "fwd_ms": [0-9.]*' $f; done
