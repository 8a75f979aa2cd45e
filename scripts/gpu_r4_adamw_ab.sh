#!/bin/bash
# Overlapped AdamW placement A/B on the 6.7B step: grid cap (default) vs a
# CU-masked side stream (32 / 64 CUs) vs no overlap; two rounds, same box.
set -o pipefail
O=gpurun_out/${OUT:-r4adamw}
mkdir -p $O
run() {  # tag, overrides
  FLEETX_BENCH_OVERRIDES="$2" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run cap128_$r ""
  run cu32_$r "Distributed.comm.overlap_optimizer_cus=32"
  run cu64_$r "Distributed.comm.overlap_optimizer_cus=64"
  run serial_$r "Distributed.comm.overlap_optimizer=False"
done
