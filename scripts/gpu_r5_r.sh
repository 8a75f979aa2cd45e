#!/bin/bash
# Round 5: 345M graph-step kernel profile; FA pairing A/B on 345M
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
for r in 1 2; do for pr in 1 0; do
  FLEETX_FA_PAIR=$pr timeout -k 10 300 python3 bench.py --model gpt-345M --steps 20 --warmup 5 > $O/b345_pair${pr}_$r.log 2>&1 || { tail -5 $O/b345_pair${pr}_$r.log; exit 1; }
  echo 345M pair=$pr $r $(grep -o '"ms_per_step": [0-9.]*' $O/b345_pair${pr}_$r.log)
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --model gpt-345M --steps 5 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window ce_stats:5:10 --steps 5 --top 40 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window ce_stats:5:10 --steps 5 --md $O/timeline.md > /dev/null
gzip -f "$f"
head -30 $O/kernels.md; head -9 $O/timeline.md
