#!/bin/bash
# 128-tile gemm5 geometry: numerics, then hipBLASLt (TN path incl. transposes)
# vs the MFMA kernel at hidden 1024 / 2048, then the 256-tile lab (regression).
set -o pipefail
O=gpurun_out/r3g128
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
for h in 1024 2048; do
  timeout -k 10 200 python tools/bench_gemm.py --hidden $h --iters 30 \
    --only fwd_x_wT,dgrad_tn_path,wgrad_tn_path,hip_fwd,hip_dgrad,hip_wgrad_f32acc > $O/bench_h$h.log 2>&1 || exit 1
done
timeout -k 10 120 tools/gemm_lab/bin/g5v_ep 5 20 > $O/lab_h4096.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py > $O/pytest_multirank.log 2>&1
echo "rc=$?" >> $O/pytest_multirank.log
