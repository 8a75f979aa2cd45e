#!/bin/bash
# Round 6: fp16 graph test after the pinned norm-plan fix; LN kernels old vs new (bench_norm)
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp16_gpu.py > $O/fp16.log 2>&1; echo "fp16 tests rc=$?"; tail -3 $O/fp16.log
for r in 1 2; do
  FLEETX_KERNELS_LIB=tools/bench_lab/_kernels_r6base.so timeout -k 10 120 python tools/bench_norm.py > $O/norm_old_$r.log 2>&1 || { echo FAIL old; tail $O/norm_old_$r.log; exit 1; }
  timeout -k 10 120 python tools/bench_norm.py > $O/norm_new_$r.log 2>&1 || { echo FAIL new; tail $O/norm_new_$r.log; exit 1; }
done
for f in $O/norm_*.log; do echo $f; grep kernel $f; done
