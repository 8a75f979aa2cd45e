#!/bin/bash
# Round 5 final: multi-rank bench rehearsals (gloo, one GPU) with the shipped vendor tuning
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5at
mkdir -p $O
port=29721
for n in 2 4 8; do
  FLEETX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --model gpt-345M \
      --steps 2 --warmup 1 > $O/reh_n$n.log 2>&1 || { echo "FAIL n=$n"; tail -30 $O/reh_n$n.log; exit 1; }
  echo "rehearse n=$n $(grep -o '"parallelism": "[a-z0-9_]*"' $O/reh_n$n.log) $(grep -o '"final_loss": [0-9.a-zA-Z]*' $O/reh_n$n.log)"
  port=$((port + 1))
done
