#!/bin/bash
# Fused column-sum finalize, wide sc1 reducer: column-sum kernel tests, model
# parity, 345M / 1.3B benches and kernel traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3cs3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_fused_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in gpt-345M gpt3-1.3B; do
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' $O/bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log) $(grep -o '"mfu": [0-9.]*' $O/bench_$m.log)" | tee -a $O/summary.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  n=$(grep -c adamw_flat "$f"); per=$((n / 5))
  python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
  gzip -f "$f"
done
