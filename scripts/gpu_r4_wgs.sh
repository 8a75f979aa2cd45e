#!/bin/bash
# Weight-gradient side stream A/B on 345M and 1.3B (interleaved).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4wgs
mkdir -p $O
run() {  # tag, env, args
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["mfu"], d["config"]["hip_graph"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run s345_$r "X=1" "--model gpt-345M --steps 20 --warmup 5"
  run s345_wgs_$r "FLEETX_BENCH_OVERRIDES=Distributed.comm.wgrad_stream=True" "--model gpt-345M --steps 20 --warmup 5"
  run b13_$r "X=1" "--model gpt3-1.3B --steps 10 --warmup 3"
  run b13_wgs_$r "FLEETX_BENCH_OVERRIDES=Distributed.comm.wgrad_stream=True" "--model gpt3-1.3B --steps 10 --warmup 3"
done
