#!/bin/bash
# Round 5: TunableOp picks for the TP2 per-rank vendor GEMMs of the multi-GPU
# bench layouts, appended to the shipped results file
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5as
mkdir -p $O
cp fleetx_amd/ops/tunableop_gfx950.csv $O/tunableop0.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv \
  timeout -k 10 600 python3 tools/tune_vendor_gemms.py > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep -c . $O/tunableop0.csv
grep "tuned M" $O/tune.log
