#!/bin/bash
# Round 5 final tree: 6.7B graph-step kernel profile (3 steady-state steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ap
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 40 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline.md > /dev/null
gzip -f "$f"
grep '"metric"' $O/prof.log | cut -c1-200
head -22 $O/kernels.md; head -9 $O/timeline.md
