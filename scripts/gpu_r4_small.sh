#!/bin/bash
# 345M / ViT-g after the tile-order autotune: routing A/B, then a 345M kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4small
mkdir -p $O
for a in wgrad wgrad,dgrad wgrad,dgrad,fwd wgrad,dgrad_act,fwd_act; do
  FLEETX_GEMM_AUTO=$a timeout -k 10 300 python bench.py --model gpt-345M --steps 20 --warmup 5 > $O/b345_$a.log 2>&1 || { tail -20 $O/b345_$a.log; exit 1; }
  echo "345M auto=$a $(tail -1 $O/b345_$a.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
done
for a in wgrad wgrad,dgrad wgrad,dgrad,fwd; do
  FLEETX_GEMM_AUTO=$a timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/vit_$a.log 2>&1 || { tail -20 $O/vit_$a.log; exit 1; }
  echo "vit auto=$a $(tail -1 $O/vit_$a.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
done
m=gpt-345M
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
python3 tools/step_timeline.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --md $O/timeline_$m.md > /dev/null
gzip -f "$f"
