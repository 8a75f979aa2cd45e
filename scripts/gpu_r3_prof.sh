#!/bin/bash
# rocprofv3 kernel traces of the 6.7B step under GEMM routing sets (same box),
# summarised over the last 3 of 5 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3prof
mkdir -p $O
for cfg in ${PROF_CFGS:-"none:" "default:wgrad,dgrad,dgrad_act,fwd_act"}; do
  tag=${cfg%%:*}; kinds=${cfg#*:}
  FLEETX_GEMM_AUTO="$kinds" timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$tag -o run -- python3 bench.py --steps 3 --warmup 2 > $O/prof_$tag.log 2>&1 || { echo "prof $tag failed"; tail -5 $O/prof_$tag.log; exit 1; }
  f=$(find $O/prof_$tag -name "*kernel_trace.csv" | head -1)
  n=$(grep -c adamw_flat "$f")
  per=$((n / 5))
  python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$tag.md > /dev/null 2>&1 || exit 1
done
