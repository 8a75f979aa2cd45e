#!/bin/bash
# Attention numerics (GPU tests) then kernel-only timings under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "flash or attention" > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
OUT=${OUT:-gpurun_out/attn} bash scripts/gpu_attn_prof.sh
