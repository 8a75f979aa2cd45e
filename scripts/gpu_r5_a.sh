#!/bin/bash
# Round 5 probe: forward GEMMs beside the overlapped AdamW (microbench), and
# the 6.7B step timeline with the forward GEMMs on gemm5 (why it loses).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py > $O/beside.jsonl 2> $O/beside.err || { tail -5 $O/beside.err; exit 1; }
cat $O/beside.jsonl
FLEETX_GEMM_AUTO=wgrad,fwd timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_fwd -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof_fwd.log 2>&1 || { tail -5 $O/prof_fwd.log; exit 1; }
f=$(find $O/prof_fwd -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 8))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((5 * per)):$((8 * per)) --steps 3 --top 30 --md $O/kernels_fwd.md > /dev/null
python3 tools/step_timeline.py "$f" --window adamw_flat:$((5 * per)):$((8 * per)) --steps 3 --md $O/timeline_fwd.md
tail -1 $O/prof_fwd.log; head -14 $O/kernels_fwd.md; head -30 $O/timeline_fwd.md
gzip -f "$f"
