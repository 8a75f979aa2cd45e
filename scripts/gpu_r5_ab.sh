#!/bin/bash
# Round 5: overlapped AdamW as few wide workgroups (1024 threads, 4 groups/lane: 4x the bytes in
# flight per CU) vs the default 128 x 256-thread cap
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ab
mkdir -p $O
for r in 1 2; do for cfg in "0 128" "1 32" "1 48" "1 64" "1 96"; do
  set -- $cfg
  FLEETX_ADAMW_OVERLAP_WIDE=$1 FLEETX_ADAMW_OVERLAP_GRID=$2 timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_w$1_g$2_$r.log 2>&1 || { tail -5 $O/b67_w$1_g$2_$r.log; exit 1; }
  echo 6.7B wide=$1 grid=$2 $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_w$1_g$2_$r.log)
done; done
