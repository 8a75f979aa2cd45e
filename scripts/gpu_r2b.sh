#!/bin/bash
# Round-2 check: optimizer semantics + fp16 attention + split-K decode, then microbenches.
set -o pipefail
mkdir -p gpurun_out/r2b
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_optim_semantics.py tests/test_kernels_gpu.py > gpurun_out/r2b/tests.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_optim.py > gpurun_out/r2b/optim.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_decode.py > gpurun_out/r2b/decode.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_decode.py --dtype fp16 >> gpurun_out/r2b/decode.log 2>&1
