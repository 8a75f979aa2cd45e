#!/bin/bash
# Forward-overlapped AdamW: root + layer 0 uncapped (they gate the first
# forward kernel) vs capped from the start; same-box A/B on 6.7B and 1.3B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3head2
mkdir -p $O
gpt() {  # model, tag, steps, env...
  local m=$1 t=$2 n=$3; shift 3
  env "$@" timeout -k 10 400 python bench.py --model $m --steps $n --warmup 3 > $O/gpt_${m}_$t.log 2>&1 || { tail -20 $O/gpt_${m}_$t.log; exit 1; }
  echo "$m $t $(grep -o '"ms_per_step": [0-9.]*' $O/gpt_${m}_$t.log) $(grep -o '"final_loss": [0-9.]*' $O/gpt_${m}_$t.log)" | tee -a $O/summary.txt
}
gpt gpt3-6.7B head2 10 FLEETX_ADAMW_OVERLAP_HEAD=2
gpt gpt3-6.7B head0 10 FLEETX_ADAMW_OVERLAP_HEAD=0
gpt gpt3-6.7B head3 10 FLEETX_ADAMW_OVERLAP_HEAD=3
gpt gpt3-6.7B head2b 10 FLEETX_ADAMW_OVERLAP_HEAD=2
gpt gpt3-1.3B head2 20 FLEETX_ADAMW_OVERLAP_HEAD=2
gpt gpt3-1.3B head0 20 FLEETX_ADAMW_OVERLAP_HEAD=0
