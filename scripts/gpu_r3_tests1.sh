#!/bin/bash
# Lab A/B of gemm5 schedule variants, then the GPU tests touched this round.
set -o pipefail
bash scripts/gpu_g5_var.sh || exit 1
O=gpurun_out/r3t1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_comm_gpu.py tests/test_model_parity_gpu.py > $O/pytest.log 2>&1
echo "rc=$?" >> $O/pytest.log
