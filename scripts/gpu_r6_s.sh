#!/bin/bash
# Round 6: ViT-g/14 same-box A/B, round-start tree vs this tree
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6s
mkdir -p $O
ROOT=$PWD
for r in 1 2; do
  for t in base new; do
    d=$ROOT; [ $t = base ] && d=$ROOT/tools/bench_lab/base
    (cd $d && timeout -k 10 400 python3 tools/bench_vit.py > $O/vit_${t}_$r.log 2>&1) || { echo "FAIL $t"; tail -5 $O/vit_${t}_$r.log; exit 1; }
    echo vit $t $r $(grep -o '"value": [0-9.]*' $O/vit_${t}_$r.log | tail -1) $(grep -o '"mfu": [0-9.]*' $O/vit_${t}_$r.log | tail -1)
  done
done
