#!/bin/bash
# Round 5: non-temporal vs cached AdamW accesses beside the forward
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ac
mkdir -p $O
for r in 1 2 3; do for nt in 1 0; do
  FLEETX_ADAMW_NT=$nt timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_nt${nt}_$r.log 2>&1 || { tail -5 $O/b67_nt${nt}_$r.log; exit 1; }
  echo 6.7B nt=$nt $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_nt${nt}_$r.log)
done; done
