#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -k "overlapped" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
