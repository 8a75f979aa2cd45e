#!/bin/bash
# Round 6 debug: fp16 fused grad norm, eager vs graph, with / without zeroed norm slots
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aj
mkdir -p $O
for m in base overlap; do
  timeout -k 10 300 python3 scripts/dbg_fp16_graph4.py $m > $O/$m.log 2>&1 || { tail -20 $O/$m.log; exit 1; }
  grep -A2 "^$m" $O/$m.log
done
