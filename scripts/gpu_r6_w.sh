#!/bin/bash
# Round 6 end: small-model steps on the final tree -- plain bench runs, then
# rocprofv3 kernel traces (3 steady steps) of GPT 345M, GPT-3 1.3B and ViT-g/14
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6w}
mkdir -p $O
for m in gpt-345M gpt3-1.3B; do
  timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > $O/b_$m.log 2>&1 || { tail -5 $O/b_$m.log; exit 1; }
  grep '"metric"' $O/b_$m.log | cut -c1-160
done
timeout -k 10 300 python3 tools/bench_vit.py --steps 10 --warmup 3 > $O/b_vit.log 2>&1 || { tail -5 $O/b_vit.log; exit 1; }
grep '"metric"' $O/b_vit.log | cut -c1-160
for m in gpt-345M gpt3-1.3B; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 5 --warmup 5 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
  python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline_$m.md > /dev/null
  rm -f "$f"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_vit -o run -- python3 tools/bench_vit.py --steps 5 --warmup 3 > $O/prof_vit.log 2>&1 || { tail -5 $O/prof_vit.log; exit 1; }
f=$(find $O/prof_vit -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window sumsq_chunks:4:7 --steps 3 --top 40 --md $O/kernels_vit.md > /dev/null
python3 tools/step_timeline.py "$f" --window sumsq_chunks:4:7 --steps 3 --md $O/timeline_vit.md > /dev/null
rm -f "$f"
head -12 $O/kernels_gpt-345M.md
