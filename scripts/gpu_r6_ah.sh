#!/bin/bash
# Round 6: attention kernel tests incl. the 8-byte row-store fallback
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6ah}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
