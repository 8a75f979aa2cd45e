#!/bin/bash
# The driver's N=1 command on the new default (graph mode), twice, plus the graph tests.
set -o pipefail
O=gpurun_out/r4drv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_graph.log 2>&1 || { tail -20 $O/pytest_graph.log; exit 1; }
tail -1 $O/pytest_graph.log
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$r.log 2>&1 || { tail -20 $O/b_$r.log; exit 1; }
  tail -1 $O/b_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' | tr '\n' ' '; echo
done
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --hip-graph 0 > $O/b_eager.log 2>&1 || { tail -20 $O/b_eager.log; exit 1; }
tail -1 $O/b_eager.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' | tr '\n' ' '; echo
