#!/bin/bash
set -o pipefail
O=gpurun_out/r3mr
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py > $O/pytest_multirank.log 2>&1
echo "rc=$?" >> $O/pytest_multirank.log
