#!/bin/bash
# Round 6: GPU suite on the current tree (+ new tests first), then LN/dropout kernels old vs new
set -o pipefail
export TMPDIR=/tmp
OUT=r6f bash scripts/gpu_r6_b.sh || exit 1
O=gpurun_out/r6f
for r in 1 2; do
  FLEETX_KERNELS_LIB=tools/bench_lab/_kernels_r6base.so timeout -k 10 120 python tools/bench_norm.py > $O/norm_old_$r.log 2>&1 || { echo FAIL old; tail $O/norm_old_$r.log; exit 1; }
  timeout -k 10 120 python tools/bench_norm.py > $O/norm_new_$r.log 2>&1 || { echo FAIL new; tail $O/norm_new_$r.log; exit 1; }
done
for f in $O/norm_*.log; do echo $f; grep kernel $f | tr '\n' ' '; echo; done
