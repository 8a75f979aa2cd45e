#!/bin/bash
# wgrad side stream "auto" default: ViT-g on/off, 1.3B default, 345M default (graph).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4wgs2
mkdir -p $O
vit() {
  timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 $2 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
}
run() {
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["mfu"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  vit vit_auto_$r ""
  vit vit_off_$r "-o Distributed.comm.wgrad_stream=False"
  run b13_auto_$r "X=1" "--model gpt3-1.3B --steps 10 --warmup 3"
  run s345_auto_$r "X=1" "--model gpt-345M --steps 20 --warmup 5"
done
