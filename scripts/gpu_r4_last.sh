#!/bin/bash
# Last check of the committed tree: smoke + the driver's N=1 command.
set -o pipefail
O=gpurun_out/r4last
mkdir -p $O
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
