#!/bin/bash
# bench.py's multi-GPU defaults rehearsed on ONE MI355X over gloo (RCCL refuses
# duplicate GPUs): N = 2 (TP2), 4 (TP2 PP2), 8 (TP2 PP2 DP2) with GPT-345M shapes.
set -o pipefail
export TMPDIR=/tmp FLEETX_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4reh
mkdir -p $OUT
port=29641
for n in 2 4 8; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --model gpt-345M \
      --steps 2 --warmup 1 > $OUT/n$n.log 2>&1 || { echo "FAIL n=$n"; tail -30 $OUT/n$n.log; exit 1; }
  echo "ok n=$n $(grep -o '"parallelism": "[a-z0-9_]*"' $OUT/n$n.log) $(grep -o '"final_loss": [0-9.]*' $OUT/n$n.log)"
  port=$((port + 1))
done
