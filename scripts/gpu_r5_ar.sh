#!/bin/bash
# Round 5: TunableOp results for the vendor GEMMs of the single-GPU model zoo
# (one shared results file), then default vs tuned on each model, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ar
mkdir -p $O
T="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv"
for m in gpt3-6.7B gpt3-1.3B gpt-345M; do
  env $T timeout -k 10 700 python3 bench.py --model $m --steps 2 --warmup 4 > $O/tune_$m.log 2>&1 || { tail -20 $O/tune_$m.log; exit 1; }
  echo "tuned $m: $(grep -c . $O/tunableop0.csv) lines"
done
env $T timeout -k 10 700 python3 tools/bench_vit.py --steps 2 --warmup 3 > $O/tune_vit.log 2>&1 || { tail -20 $O/tune_vit.log; exit 1; }
echo "tuned vit: $(grep -c . $O/tunableop0.csv) lines"
cp $O/tunableop0.csv fleetx_amd/ops/tunableop_gfx950.csv
for r in 1 2; do
  for v in off on; do
    for m in gpt3-6.7B gpt-345M; do
      FLEETX_VENDOR_TUNE=$v timeout -k 10 400 python3 bench.py --model $m --steps 10 --warmup 4 > $O/b_${m}_${v}_$r.log 2>&1 || { tail -5 $O/b_${m}_${v}_$r.log; exit 1; }
      echo "$m vendor_tune=$v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${m}_${v}_$r.log)" | tee -a $O/summary.txt
    done
    FLEETX_VENDOR_TUNE=$v timeout -k 10 400 python3 tools/bench_vit.py --steps 10 --warmup 3 > $O/vit_${v}_$r.log 2>&1 || { tail -5 $O/vit_${v}_$r.log; exit 1; }
    echo "ViT-g vendor_tune=$v run $r $(grep -o '"value": [0-9.]*' $O/vit_${v}_$r.log | tail -1)" | tee -a $O/summary.txt
  done
done
