#!/bin/bash
# Round 6: fp16 graph determinism probe, then new / changed GPU tests, full suite, smoke, FA lab
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
REPS=2 timeout -k 10 200 python scripts/dbg_fp16_graph.py > $O/dbg.log 2>&1 || { echo "FAIL dbg"; tail -20 $O/dbg.log; exit 1; }
grep -v "WARNING\|INFO" $O/dbg.log | tail -12
bash scripts/gpu_r6_b.sh
