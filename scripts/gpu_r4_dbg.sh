#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4dbg
mkdir -p $O
T=tests/test_kernels_gpu.py::test_forward_overlapped_adamw_matches_serial
timeout -k 10 200 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > $O/alone.log 2>&1; echo "alone rc=$?"; tail -1 $O/alone.log
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py $T -q --timeout 120 --timeout-method thread > $O/after_gemm.log 2>&1; echo "after_gemm rc=$?"; tail -1 $O/after_gemm.log
timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py $T -q --timeout 120 --timeout-method thread > $O/after_comm.log 2>&1; echo "after_comm rc=$?"; tail -1 $O/after_comm.log
