#!/bin/bash
# Round 5: PyTorch TunableOp over the vendor GEMMs (hipBLASLt / rocBLAS
# solutions timed per shape) on the 6.7B step: tune once, then default vs
# tuned, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5aq
mkdir -p $O
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv \
  timeout -k 10 700 python3 bench.py --steps 3 --warmup 4 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep '"metric"' $O/tune.log | cut -c1-200
ls -la $O
for r in 1 2; do
  for v in def tuned; do
    if [ $v = tuned ]; then e="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv"; else e=""; fi
    env $e timeout -k 10 400 python3 bench.py --steps 10 --warmup 4 > $O/b67_${v}_$r.log 2>&1 || { tail -5 $O/b67_${v}_$r.log; exit 1; }
    echo "6.7B $v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_${v}_$r.log)" | tee -a $O/summary.txt
  done
done
