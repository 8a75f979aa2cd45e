#!/bin/bash
# GEMM numerics + micro-benchmark on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gemm.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_gemm.py --iters 20 --variants ${GEMM_VARIANTS:-0,1} --only ${GEMM_CASES:-fwd_x_wT,dgrad_tn_path,wgrad_tn_path,hip_fwd,hip_fwd_gelu,hip_dgrad,hip_dgrad_dgelu,hip_wgrad_f32acc} > gpurun_out/bench_gemm.log 2>&1
rc=$?
cat gpurun_out/bench_gemm.log | grep -v amdgpu.ids
exit $rc
