#!/bin/bash
# 345M and 1.3B: bench, then a kernel trace with the step timeline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3small
mkdir -p $O
for m in gpt-345M gpt3-1.3B; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  n=$(grep -c adamw_flat "$f"); per=$((n / 5))
  python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
  python3 tools/step_timeline.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --md $O/timeline_$m.md > /dev/null
  gzip -f "$f"
done
