#!/bin/bash
# Host-overhead changes (cached AdamW launch args, one-launch fused norm):
# GPU tests that cover them, then 6.7B / 1.3B / 345M benches.
set -o pipefail
O=gpurun_out/r3host
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_fused_norm_gpu.py tests/test_graph_gpu.py tests/test_fp16_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in gpt3-6.7B gpt3-1.3B gpt-345M; do
  st=20; [ $m = gpt3-6.7B ] && st=10
  timeout -k 10 400 python bench.py --model $m --steps $st --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' $O/bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log) $(grep -o '"mfu": [0-9.]*' $O/bench_$m.log)" | tee -a $O/summary.txt
done
