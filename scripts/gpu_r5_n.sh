#!/bin/bash
# Round 5: multi-rank suite (overlap tests), bench.py multi-GPU rehearsal over gloo,
# 6.7B default profile, small-model benches with bf16 gradients
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_mr.log 2>&1 || { tail -40 $O/pytest_mr.log; exit 1; }
tail -1 $O/pytest_mr.log
port=29651
for n in 2 4 8; do
  FLEETX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --model gpt-345M \
      --steps 2 --warmup 1 > $O/reh_n$n.log 2>&1 || { echo "FAIL n=$n"; tail -30 $O/reh_n$n.log; exit 1; }
  echo "ok n=$n $(grep -o '"parallelism": "[a-z0-9_]*"' $O/reh_n$n.log) $(grep -o '"final_loss": [0-9.]*' $O/reh_n$n.log)"
  port=$((port + 1))
done
for m in gpt-345M gpt3-1.3B; do
  timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > $O/bench_$m.log 2>&1 || { tail -5 $O/bench_$m.log; exit 1; }
  echo $m $(grep -o '"value": [0-9.]*' $O/bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log) $(grep -o '"mfu": [0-9.]*' $O/bench_$m.log)
done
timeout -k 10 400 python3 tools/bench_vit.py > $O/bench_vit.log 2>&1 || { tail -5 $O/bench_vit.log; exit 1; }
tail -2 $O/bench_vit.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 30 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline.md > /dev/null
gzip -f "$f"
grep -o '"ms_per_step": [0-9.]*' $O/prof.log
