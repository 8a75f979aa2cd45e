#!/bin/bash
# Round 5: chunked LM head + cross entropy (no logits tensor) vs materialised logits, 6.7B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ag
mkdir -p $O
for r in 1 2; do for f in False True; do
  FLEETX_BENCH_OVERRIDES="Model.fused_lm_head_ce=$f" timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_f${f}_$r.log 2>&1 || { tail -5 $O/b67_f${f}_$r.log; exit 1; }
  echo 6.7B fused_head_ce=$f $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_f${f}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b67_f${f}_$r.log) $(grep -o '"peak_mem_gb": [0-9.]*' $O/b67_f${f}_$r.log)
done; done
