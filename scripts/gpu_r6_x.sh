#!/bin/bash
# Round 6: flash attention fwd/bwd rates vs sequence length, causal / dropout
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6x}
mkdir -p $O
for cfg in "8 1024 32 128" "4 2048 32 128" "2 4096 32 128" "8 1024 16 64"; do
  set -- $cfg
  timeout -k 10 200 python3 tools/bench_attention.py --b $1 --s $2 --h $3 --d $4 --iters 30 >> $O/attn.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
cat $O/attn.jsonl
