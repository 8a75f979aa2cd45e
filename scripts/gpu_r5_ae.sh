#!/bin/bash
# Round 5: ViT-g forward GEMMs on gemm5 (persistent, XCD rectangles), with / without the overlapped update
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ae
mkdir -p $O
for r in 1 2; do
  for cfg in "wgrad True" "wgrad,fwd True" "wgrad,fwd False" "wgrad False"; do
    set -- $cfg
    FLEETX_GEMM_AUTO=$1 timeout -k 10 300 python3 tools/bench_vit.py -o Distributed.comm.overlap_optimizer=$2 > $O/vit_${1}_$2_$r.log 2>&1 || { tail -5 $O/vit_${1}_$2_$r.log; exit 1; }
    echo vit auto=$1 overlap=$2 $r $(grep -o '"value": [0-9.]*' $O/vit_${1}_$2_$r.log | tail -1)
  done
done
