#!/bin/bash
# Round 6: model zoo on the current tree (same box): 345M, 1.3B, ViT-g, 175B-shape 4 layers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6m
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  echo $name $(grep -o '"value": [0-9.]*' $O/$name.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log) $(grep -o '"mfu": [0-9.]*' $O/$name.log) $(grep -o '"peak_mem_gb": [0-9.]*' $O/$name.log)
}
run b345 --model gpt-345M --steps 20 --warmup 5
run b13 --model gpt3-1.3B --steps 20 --warmup 5
timeout -k 10 400 python3 tools/bench_vit.py > $O/vit.log 2>&1 || { tail -5 $O/vit.log; exit 1; }
echo vit $(grep -o '"value": [0-9.]*' $O/vit.log | tail -1) $(grep -o '"mfu": [0-9.]*' $O/vit.log | tail -1)
run b175_4L --model gpt3-175B-4L --steps 10 --warmup 3
