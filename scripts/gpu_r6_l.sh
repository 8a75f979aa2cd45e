#!/bin/bash
# Round 6: multi-rank rehearsals over gloo on one GPU (HIP kernels), bench.py default
# layouts N=1/2/4/8 at GPT-345M shapes (16-bit gradient storage now also under 1F1B /
# accumulation), plus the N=8 config-3 layout with fp32 gradient storage for comparison
set -o pipefail
export TMPDIR=/tmp FLEETX_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 300 python3 bench.py --model gpt-345M --steps 2 --warmup 1 --hip-graph 0 > $O/n1.log 2>&1 || { echo FAIL n1; tail -20 $O/n1.log; exit 1; }
echo "n=1 $(grep -o '"parallelism": "[a-z0-9_]*"' $O/n1.log) $(grep -o '"final_loss": [0-9.]*' $O/n1.log)"
port=29731
for n in 2 4 8; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --model gpt-345M \
      --steps 2 --warmup 1 > $O/n$n.log 2>&1 || { echo "FAIL n=$n"; tail -30 $O/n$n.log; exit 1; }
  echo "n=$n $(grep -o '"parallelism": "[a-z0-9_]*"' $O/n$n.log) $(grep -o '"final_loss": [0-9.]*' $O/n$n.log) $(grep -o '"grad_reduce_dtype": "[a-z0-9]*"' $O/n$n.log)"
  port=$((port + 1))
done
FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=float32" timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --model gpt-345M \
    --steps 2 --warmup 1 > $O/n8_g32.log 2>&1 || { echo "FAIL n8 g32"; tail -30 $O/n8_g32.log; exit 1; }
echo "n=8 fp32-grads $(grep -o '"final_loss": [0-9.]*' $O/n8_g32.log)"
grep -h "16-bit\|grad storage\|grad_dtype" $O/n8.log | head -3
