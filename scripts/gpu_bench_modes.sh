#!/bin/bash
# 6.7B 1-GPU bench under each GEMM routing mode (FLEETX_GEMM=blas|auto|hip).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for mode in ${MODES:-blas auto hip}; do
  echo "== FLEETX_GEMM=$mode"
  FLEETX_GEMM=$mode timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench_$mode.log 2>&1
  rc=$?
  tail -1 gpurun_out/bench_$mode.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$mode.log; exit $rc; fi
done
