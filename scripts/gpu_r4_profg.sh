#!/bin/bash
# Kernel trace of the shipped 6.7B default (whole-step graph) with its timeline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4profg
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 8))
echo "adamw launches $n per-step $per"
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((5 * per)):$((8 * per)) --steps 3 --top 40 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window adamw_flat:$((5 * per)):$((8 * per)) --steps 3 --md $O/timeline.md
head -12 $O/kernels.md; head -10 $O/timeline.md
