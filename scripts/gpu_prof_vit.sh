#!/bin/bash
# rocprofv3 kernel trace of the ViT-g/14 training step (tools/bench_vit.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prof_vit}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 tools/bench_vit.py --steps 4 --warmup 2 $VIT_ARGS > $OUT/bench.log 2>&1 || { echo "prof failed"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-200
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --steps 6 --top 30 --md $OUT/kernels.md > /dev/null 2>&1
head -32 $OUT/kernels.md
