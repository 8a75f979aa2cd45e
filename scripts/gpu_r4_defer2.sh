#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4defer2
mkdir -p $O
run() {
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["mfu"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run serial_$r "FLEETX_BENCH_OVERRIDES=Distributed.comm.overlap_optimizer=False" "--model gpt-345M --steps 20 --warmup 5"
  for g in 128 256 512 0; do
    run defer_g${g}_$r "FLEETX_ADAMW_OVERLAP_GRID=$g" "--model gpt-345M --steps 20 --warmup 5"
  done
done
