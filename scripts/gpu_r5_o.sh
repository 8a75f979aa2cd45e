#!/bin/bash
# Round 5: tp2_pp2 (n=4) rehearsal NaN hunt
set -o pipefail
export TMPDIR=/tmp FLEETX_DIST_BACKEND=gloo
O=gpurun_out/r5o
mkdir -p $O
port=29661
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 4 --model gpt-345M \
      --steps 2 --warmup 1 > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }
  echo "$name $(grep -o '"final_loss": [0-9.a-zA-Z]*' $O/$name.log)"
  port=$((port + 1))
}
run base X=1
run noovl FLEETX_BENCH_OVERRIDES=Distributed.comm.overlap_optimizer=False
run nofnorm FLEETX_BENCH_OVERRIDES=Distributed.comm.fused_grad_norm=False
run nows FLEETX_BENCH_OVERRIDES=Distributed.comm.wgrad_stream=False
run nooneshot FLEETX_ONESHOT=0
