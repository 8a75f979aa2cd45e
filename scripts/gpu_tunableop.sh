#!/bin/bash
# Tune every hipBLASLt/rocBLAS GEMM of the 6.7B step with PyTorch TunableOp, then
# re-run the bench reading the tuned table (tuning off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tunable
mkdir -p $O
export PYTHONUNBUFFERED=1
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-15} PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=256
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 > $O/tune.log 2>&1 &&
ls -la $O && PYTORCH_TUNABLEOP_VERBOSE=0 PYTORCH_TUNABLEOP_TUNING=0 \
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_tuned.log 2>&1 &&
tail -1 $O/bench_tuned.log
