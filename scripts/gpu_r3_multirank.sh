#!/bin/bash
# Multi-rank GPU equivalence (2 ranks sharing the GPU) with the fused gradient
# norm now on by default: every layout vs the single-rank curve.
set -o pipefail
O=gpurun_out/r3mr
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --tb=short --timeout 300 --timeout-method thread \
  tests/test_multirank_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit 1
