#!/bin/bash
# Multi-rank checks after the LayerNorm / split-K changes: the 2-rank GPU
# equivalence suite (every layout vs the single-rank run), then the 8-rank
# gloo rehearsal of bench.py --gpus 8 (config-3 default layout, ZeRO-1, planner).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3mr2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --tb=short --timeout 300 --timeout-method thread \
  tests/test_multirank_gpu.py tests/test_kernels_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 1000 bash tools/rehearse_hybrid8_gpu.sh > $O/rehearse8.log 2>&1
rc=$?; tail -5 $O/rehearse8.log; exit $rc
