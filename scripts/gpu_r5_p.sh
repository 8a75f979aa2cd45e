#!/bin/bash
# Round 5: gloo p2p staged through host (rehearsal NaN), 345M grad16 A/B, ViT epilogue A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
port=29671
run() {  # name, nranks, env...
  local name=$1 n=$2; shift 2
  env FLEETX_DIST_BACKEND=gloo "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --model gpt-345M \
      --steps 2 --warmup 1 > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }
  echo "$name $(grep -o '"final_loss": [0-9.a-zA-Z]*' $O/$name.log)"
  port=$((port + 1))
}
run n4a 4 X=1
run n4b 4 X=1
run n4c 4 FLEETX_BENCH_OVERRIDES=Distributed.comm.overlap_optimizer=False
run n8 8 X=1
for r in 1 2; do for g in bfloat16 float32; do
  FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=$g" timeout -k 10 300 python3 bench.py --model gpt-345M --steps 20 --warmup 5 > $O/b345_${g}_$r.log 2>&1 || { tail -5 $O/b345_${g}_$r.log; exit 1; }
  echo 345M $g $r $(grep -o '"ms_per_step": [0-9.]*' $O/b345_${g}_$r.log)
done; done
for r in 1 2; do for v in wgrad wgrad,fwd_act,dgrad_act; do
  FLEETX_GEMM_AUTO=$v timeout -k 10 300 python3 tools/bench_vit.py > $O/vit_${v}_$r.log 2>&1 || { tail -5 $O/vit_${v}_$r.log; exit 1; }
  echo vit $v $r $(grep -o '"value": [0-9.]*' $O/vit_${v}_$r.log | tail -1)
done; done
