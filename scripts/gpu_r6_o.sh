#!/bin/bash
# Round 6: ZeRO-1 with 16-bit gradient storage -- multirank GPU tests and an 8-rank ZeRO-1
# rehearsal (gloo on one GPU)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multirank_gpu.py > $O/mr.log 2>&1 || { echo FAIL; tail -30 $O/mr.log; exit 1; }
tail -1 $O/mr.log
port=29771
for lay in "1,1,1,8,8,1" "2,2,2,4"; do
  FLEETX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --model gpt-345M \
      --steps 2 --warmup 1 --layout $lay > $O/reh_$lay.log 2>&1 || { echo "FAIL $lay"; tail -30 $O/reh_$lay.log; exit 1; }
  echo "layout $lay $(grep -o '"parallelism": "[a-z0-9_]*"' $O/reh_$lay.log) $(grep -o '"final_loss": [0-9.]*' $O/reh_$lay.log)"
  port=$((port + 1))
done
