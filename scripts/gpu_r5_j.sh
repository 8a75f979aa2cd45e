#!/bin/bash
# Round 5: kernel traces of the 6.7B step, bf16 vs fp32 gradient storage
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
for g in bfloat16 float32; do
FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=$g" timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$g -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof_$g.log 2>&1 || { tail -5 $O/prof_$g.log; exit 1; }
f=$(find $O/prof_$g -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 25 --md $O/kernels_$g.md > /dev/null
python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline_$g.md > /dev/null
grep -o '"ms_per_step": [0-9.]*' $O/prof_$g.log; head -16 $O/kernels_$g.md
gzip -f "$f"
done
