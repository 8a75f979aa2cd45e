#!/bin/bash
# 8-rank rehearsal on ONE MI355X over gloo (RCCL refuses duplicate GPUs):
# bench.py --gpus 8 with its DEFAULT layout (BASELINE config 3: TP2 x PP2 x DP2,
# 1F1B, micro-batches, embedding all-reduce, vocab-parallel CE; the JSON line
# must say "parallelism": "dp2_tp2_pp2"), a pinned ZeRO-1 layout and the
# planner's 8-GPU choice, each with the HIP kernels.  GPT-345M shapes keep 8 copies within one device; not a
# performance run (gloo moves every collective through host memory).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp FLEETX_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/rehearse8
mkdir -p $OUT
port=29631
for layout in default "1,1,1,8,8,1" "planner"; do
  arg=""
  [ "$layout" != default ] && arg="--layout $layout"
  tag=$(echo "$layout" | tr ',' '_')
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --model gpt-345M \
      --steps 2 --warmup 1 $arg > $OUT/$tag.log 2>&1 || { echo "FAIL $layout"; tail -30 $OUT/$tag.log; exit 1; }
  echo "ok $layout $(grep -o '"parallelism": "[a-z0-9_]*"' $OUT/$tag.log) $(grep -o '"final_loss": [0-9.]*' $OUT/$tag.log)"
  port=$((port + 1))
done
