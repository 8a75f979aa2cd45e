#!/bin/bash
# Weight-gradient side stream inside the whole-step graph: 1.3B and 6.7B, interleaved.
set -o pipefail
O=gpurun_out/r4wgsg
mkdir -p $O
for r in 1 2; do
  for w in False True; do
    FLEETX_BENCH_OVERRIDES="Distributed.comm.wgrad_stream=$w" timeout -k 10 300 python3 bench.py --model gpt3-1.3B --steps 20 --warmup 5 > $O/b13_${w}_$r.log 2>&1 || { tail -20 $O/b13_${w}_$r.log; exit 1; }
    echo "1.3B wgrad_stream=$w run $r: $(tail -1 $O/b13_${w}_$r.log | grep -o '"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' | tr '\n' ' ')" | tee -a $O/summary.txt
  done
done
for r in 1 2; do
  for w in False True; do
    FLEETX_BENCH_OVERRIDES="Distributed.comm.wgrad_stream=$w" timeout -k 10 400 python3 bench.py --steps 10 --warmup 5 > $O/b67_${w}_$r.log 2>&1 || { tail -20 $O/b67_${w}_$r.log; exit 1; }
    echo "6.7B wgrad_stream=$w run $r: $(tail -1 $O/b67_${w}_$r.log | grep -o '"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
  done
done
