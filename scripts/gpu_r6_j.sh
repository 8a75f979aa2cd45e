#!/bin/bash
# Round 6: 6.7B graph-step kernel profiles (3 steady steps), bf16 and fp16 O2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6j}
mkdir -p $O
for dt in ${DTS:-bf16 fp16}; do
  ov=""; [ $dt = fp16 ] && ov="Engine.mix_precision.dtype=float16"
  FLEETX_BENCH_OVERRIDES=$ov timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$dt -o run -- python3 bench.py --steps 5 --warmup 5 > $O/prof_$dt.log 2>&1 || { tail -5 $O/prof_$dt.log; exit 1; }
  f=$(find $O/prof_$dt -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 40 --md $O/kernels_$dt.md > /dev/null
  python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline_$dt.md > /dev/null
  gzip -f "$f"
  grep '"metric"' $O/prof_$dt.log | cut -c1-200
done
