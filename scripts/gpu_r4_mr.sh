#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4mr
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_comm_gpu.py tests/test_model_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -40; tail -2 $O/pytest.log; exit $rc
