#!/bin/bash
# Round 6: gemm5 K-loop schedules (4 vs 2 barriers per K-tile) on the 6.7B shapes,
# standalone lab binaries (tools/gemm_lab/build_g5_var.sh), output hashes compared
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
for r in 1 2; do
  for v in base b2 b2s0 b2g3 b2p4; do
    LAB_HASH=1 timeout -k 10 90 tools/gemm_lab/bin/g5v_$v 5 20 > $O/${v}_$r.log 2>&1 || { echo "FAIL $v rc=$?"; tail -5 $O/${v}_$r.log; exit 1; }
    echo "$v $r done"
  done
done
