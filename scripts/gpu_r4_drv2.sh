#!/bin/bash
# Driver command on the new defaults (graph, capped deferred update for 6.7B), 345M default, graph tests.
set -o pipefail
O=gpurun_out/r4drv2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_graph.log 2>&1 || { tail -20 $O/pytest_graph.log; exit 1; }
tail -1 $O/pytest_graph.log
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b67_$r.log 2>&1 || { tail -20 $O/b67_$r.log; exit 1; }
  tail -1 $O/b67_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' | tr '\n' ' '; echo
done
timeout -k 10 300 python3 bench.py --model gpt-345M --steps 20 --warmup 5 > $O/b345.log 2>&1 || { tail -20 $O/b345.log; exit 1; }
tail -1 $O/b345.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' '; echo
