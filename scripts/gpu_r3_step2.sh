#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3step2
mkdir -p $O
timeout -k 10 120 tools/gemm_lab/bin/g5v_ep 5 20 > $O/lab_ep.log 2>&1 || exit 1
for cfg in "none:" "wgrad:wgrad" "default:wgrad,dgrad" "none2:" "default2:wgrad,dgrad"; do
  tag=${cfg%%:*}; kinds=${cfg#*:}
  FLEETX_GEMM_AUTO="$kinds" timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/bench_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $O/bench_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.log)" | tee -a $O/summary.txt
done
PROF_CFGS="default:wgrad,dgrad" bash scripts/gpu_r3_prof.sh
