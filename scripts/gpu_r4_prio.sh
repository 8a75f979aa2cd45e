#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4prio
mkdir -p $O
python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())" 2>&1 | tail -1
run() {
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run base_$r "X=1" "--steps 10 --warmup 3"
  run stephi_$r "FLEETX_STEP_STREAM_PRIORITY=-1" "--steps 10 --warmup 3"
  run sidehi_$r "FLEETX_SIDE_STREAM_PRIORITY=-1" "--steps 10 --warmup 3"
done
