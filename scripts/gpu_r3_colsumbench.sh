#!/bin/bash
# Column-sum kernel bandwidth vs workgroups per reduction (tools/bench_colsum.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3csb
mkdir -p $O
for b in 256 512 1024 2048 4096; do
  FLEETX_COLSUM_BLOCKS=$b timeout -k 10 120 python tools/bench_colsum.py >> $O/colsum.jsonl 2> $O/err_$b.log || { tail -5 $O/err_$b.log; exit 1; }
done
cat $O/colsum.jsonl
