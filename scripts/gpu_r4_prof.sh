#!/bin/bash
# Kernel traces + timelines of 345M, 1.3B and 6.7B with the round-4 defaults.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4prof
mkdir -p $O
for m in gpt-345M gpt3-1.3B gpt3-6.7B; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  n=$(grep -c adamw_flat "$f"); per=$((n / 5))
  python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
  python3 tools/step_timeline.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --md $O/timeline_$m.md > /dev/null
  gzip -f "$f"
done
head -25 $O/kernels_gpt-345M.md
