#!/bin/bash
# ViT-g/14: whole-step HIP graph (deferred AdamW, cap 128 / uncapped) vs eager, interleaved.
set -o pipefail
O=gpurun_out/r4vitg
mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 > $O/eager_$r.log 2>&1 || { tail -20 $O/eager_$r.log; exit 1; }
  echo "eager run $r: $(tail -1 $O/eager_$r.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
  timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 -o Engine.cuda_graph=True > $O/graph_$r.log 2>&1 || { tail -20 $O/graph_$r.log; exit 1; }
  echo "graph run $r: $(tail -1 $O/graph_$r.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
  FLEETX_ADAMW_OVERLAP_GRID=0 timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 -o Engine.cuda_graph=True > $O/graph0_$r.log 2>&1 || { tail -20 $O/graph0_$r.log; exit 1; }
  echo "graph uncapped run $r: $(tail -1 $O/graph0_$r.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
done
grep -i "cuda_graph\|graph disabled" $O/graph_1.log | head -3
