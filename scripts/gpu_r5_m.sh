#!/bin/bash
# Round 5: ZeRO-1/2 overlapped update + gather (bitwise vs serial), SP dgrad on the GEMM plan,
# full multi-rank suite; default-step kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_mr.log 2>&1 || { tail -40 $O/pytest_mr.log; exit 1; }
tail -3 $O/pytest_mr.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 30 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline.md > /dev/null
gzip -f "$f"
grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus[^,]*, "steps[^,]*, "warmup[^,]*, "ms_per_step": [0-9.]*' $O/prof.log
head -20 $O/kernels.md
