#!/bin/bash
# Per-kernel split of the stored-dS vs recompute attention backward (D128 causal and D64).
# (ran with profiles/r4_ds/stored_ds.patch applied; FLEETX_FA_BWD_DS was not kept)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4dsprof
mkdir -p $O
for f in 1 0; do
  FLEETX_FA_BWD_DS=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$f -o run -- python3 tools/bench_attention.py --iters 20 > $O/log$f.txt 2>&1 || exit 1
done
for f in 1 0; do echo "== ds$f"; find $O/p$f -name "*kernel_stats.csv" -exec head -12 {} \; ; done
