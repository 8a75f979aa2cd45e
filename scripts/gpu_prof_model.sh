#!/bin/bash
# rocprofv3 kernel trace of bench.py for one model (MODEL env), summarised per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODEL=${MODEL:-gpt-345M}
OUT=${OUT:-gpurun_out/prof_$MODEL}; mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --model $MODEL --steps 5 --warmup 3 > $OUT/bench.log 2>&1 || { echo "prof failed"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-200
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --steps 8 --top 40 --md $OUT/kernels.md > /dev/null 2>&1
head -42 $OUT/kernels.md
