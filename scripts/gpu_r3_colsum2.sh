#!/bin/bash
# Fused column-sum finalize: kernel / model / engine
# GPU tests, then the three benches and a 345M kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3cs2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_fused_norm_gpu.py \
  tests/test_graph_gpu.py tests/test_fp16_gpu.py tests/test_decode_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in gpt-345M gpt3-1.3B gpt3-6.7B; do
  st=20; [ $m = gpt3-6.7B ] && st=10
  timeout -k 10 400 python bench.py --model $m --steps $st --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' $O/bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log) $(grep -o '"mfu": [0-9.]*' $O/bench_$m.log)" | tee -a $O/summary.txt
done
for m in gpt-345M gpt3-1.3B; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
gzip -f "$f"
done
