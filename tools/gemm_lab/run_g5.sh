set -o pipefail
mkdir -p gpurun_out/g5
FLEETX_GEMM_PF=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/g5/pytest_pf5.log 2>&1
echo "pytest rc=$?" >> gpurun_out/g5/pytest_pf5.log
timeout -k 10 120 tools/gemm_lab/bin/gemm_lab_abl0 5 20 > gpurun_out/g5/lab_v5.log 2>&1 && timeout -k 10 120 tools/gemm_lab/bin/gemm_lab_abl0 0 20 > gpurun_out/g5/lab_v0.log 2>&1
