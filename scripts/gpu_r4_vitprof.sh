#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4vit
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/bench_vit.py --steps 4 --warmup 2 > $O/bench.log 2>&1 || { echo "prof failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 6))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((6 * per)) --steps 4 --top 40 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window adamw_flat:$((2 * per)):$((6 * per)) --steps 4 --md $O/timeline.md > /dev/null
gzip -f "$f"
head -40 $O/kernels.md; head -10 $O/timeline.md
