#!/bin/bash
# Column-sum kernels with 4 rows' loads in flight: kernel tests, then 6.7B and
# 345M kernel traces (per-call times of coltile_partial / dropout_bwd_colsum).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3rows4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_fused_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in gpt3-6.7B gpt-345M; do
  timeout -k 10 400 python bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log)" | tee -a $O/summary.txt
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  n=$(grep -c adamw_flat "$f"); per=$((n / 5))
  python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
  gzip -f "$f"
done
