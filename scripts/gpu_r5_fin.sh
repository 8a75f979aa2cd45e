#!/bin/bash
# Round 5 final numbers: model zoo benches, fp16, 175B-shape, ViT-g, multi-rank rehearsal
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5fin}
mkdir -p $O
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  echo $name $(grep -o '"value": [0-9.]*' $O/$name.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log) $(grep -o '"mfu": [0-9.]*' $O/$name.log) $(grep -o '"peak_mem_gb": [0-9.]*' $O/$name.log)
}
run b67_1 --steps 20 --warmup 5
run b67_2 --steps 20 --warmup 5
FLEETX_BENCH_OVERRIDES="Engine.mix_precision.dtype=float16" run b67_fp16 --steps 10 --warmup 5
run b13 --model gpt3-1.3B --steps 20 --warmup 5
run b345 --model gpt-345M --steps 20 --warmup 5
run b175_4L --model gpt3-175B-4L --steps 10 --warmup 3
timeout -k 10 400 python3 tools/bench_vit.py > $O/vit.log 2>&1 || { tail -5 $O/vit.log; exit 1; }
echo vit $(grep -o '"value": [0-9.]*' $O/vit.log | tail -1) $(grep -o '"mfu": [0-9.]*' $O/vit.log | tail -1)
port=29691
for n in 2 4 8; do
  FLEETX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --model gpt-345M \
      --steps 2 --warmup 1 > $O/reh_n$n.log 2>&1 || { echo "FAIL n=$n"; tail -30 $O/reh_n$n.log; exit 1; }
  echo "rehearse n=$n $(grep -o '"parallelism": "[a-z0-9_]*"' $O/reh_n$n.log) $(grep -o '"final_loss": [0-9.a-zA-Z]*' $O/reh_n$n.log)"
  port=$((port + 1))
done
