#!/bin/bash
# Benches (6.7B / 1.3B / 345M) and a rocprofv3 kernel-stats pass of the 6.7B step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r2d}; mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gpt3-6.7B gpt3-1.3B gpt-345M; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 > $OUT/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 $OUT/bench_$m.log; exit 1; }
  grep '^{' $OUT/bench_$m.log | cut -c1-300
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window adamw_flat:132:330 --steps 3 --top 32 --md $OUT/kernels_6.7B.md > /dev/null 2>&1
head -34 $OUT/kernels_6.7B.md
