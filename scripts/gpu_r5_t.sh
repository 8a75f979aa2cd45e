#!/bin/bash
# Round 5: full GPU suite + smoke + default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-300
FLEETX_FA_DKDV_W8=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 200 --timeout-method thread > $O/pytest_w8.log 2>&1 || { tail -30 $O/pytest_w8.log; exit 1; }
tail -1 $O/pytest_w8.log
for r in 1 2; do for w in 0 1; do
  FLEETX_FA_DKDV_W8=$w timeout -k 10 120 python3 tools/bench_attention.py --iters 50 > $O/attn_w8${w}_$r.jsonl 2>&1 || { tail -5 $O/attn_w8${w}_$r.jsonl; exit 1; }
  echo w8=$w; grep '"causal": true' $O/attn_w8${w}_$r.jsonl | grep -o '"dropout": [0-9.]*, "fwd_ms[^}]*'
done; done
