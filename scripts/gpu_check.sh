#!/bin/bash
# GPU-box check: kernel tests, smoke, then a short bench.  Stops on any crash
# (exit codes other than 0/1 from pytest), never retries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 2"}
timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?
tail -5 gpurun_out/bench.log
exit $rc
