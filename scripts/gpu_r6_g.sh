#!/bin/bash
# Round 6: re-run the tests that failed in r6f, then the LN/dropout kernel A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad_16bit" "tests/test_multirank_gpu.py::test_layout_matches_single_rank_on_gpu" "tests/test_multirank_gpu.py::test_rccl_collective_forms_on_gpu" "tests/test_multirank_gpu.py::test_tp_oneshot_allreduce_matches_single_rank" > $O/t.log 2>&1 || { echo FAIL; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
FLEETX_KERNELS_LIB=$(ls tools/fa_lab/_kernels*.so) timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tools/fa_lab/test_fa_wave64_lab.py > $O/fa_lab.log 2>&1 || { echo "FAIL fa_lab"; tail -30 $O/fa_lab.log; exit 1; }
tail -1 $O/fa_lab.log
for r in 1 2; do
  FLEETX_KERNELS_LIB=tools/bench_lab/_kernels_r6base.so timeout -k 10 120 python tools/bench_norm.py > $O/norm_old_$r.log 2>&1 || { echo FAIL old; tail $O/norm_old_$r.log; exit 1; }
  timeout -k 10 120 python tools/bench_norm.py > $O/norm_new_$r.log 2>&1 || { echo FAIL new; tail $O/norm_new_$r.log; exit 1; }
done
for f in $O/norm_*.log; do echo $f; grep kernel $f | tr '\n' ' '; echo; done
