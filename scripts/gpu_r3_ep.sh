#!/bin/bash
set -o pipefail
bash scripts/gpu_g5_var.sh || exit 1
O=gpurun_out/r3ep
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest.log 2>&1
echo "rc=$?" >> $O/pytest.log
