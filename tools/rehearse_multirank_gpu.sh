#!/bin/bash
# Multi-rank rehearsal on ONE MI355X: 2 ranks share the device over gloo
# (RCCL refuses duplicate GPUs), exercising the distributed engine paths
# (ZeRO-1 bucketed reductions + overlapped param gather, DP, TP, PP) with
# device tensors, async collectives and side streams.  Not a performance run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp FLEETX_DIST_BACKEND=gloo
OUT=gpurun_out/rehearse
mkdir -p $OUT
port=29531
for layout in planner "2,1,1,8" "1,2,1,8" "1,1,2,4" "1,1,1,8,2,2"; do
  arg=""
  [ "$layout" != planner ] && arg="--layout $layout"
  tag=$(echo "$layout" | tr ',' '_')
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --model gpt3-1.3B \
      --steps 3 --warmup 1 $arg > $OUT/$tag.log 2>&1 || { echo "FAIL $layout"; tail -20 $OUT/$tag.log; exit 1; }
  echo "ok $layout $(tail -1 $OUT/$tag.log | cut -c1-40) $(grep -o '"final_loss": [0-9.]*' $OUT/$tag.log)"
  port=$((port + 1))
done
