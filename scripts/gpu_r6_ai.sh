#!/bin/bash
# Round 6 end, last tree: full GPU suite, smoke, driver-K/W bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6final4
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_20.log 2>&1 || { tail -5 $O/bench_20.log; exit 1; }
grep '"metric"' $O/bench_20.log | cut -c1-200
