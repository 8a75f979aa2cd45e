#!/bin/bash
# Round 6 end (second pass, after the attention store change): full GPU suite,
# smoke, FA lab tests, default bench x2, 6.7B kernel profile
set -o pipefail
export TMPDIR=/tmp
OUT=r6final2 bash scripts/gpu_r6_final.sh || exit 1
O=gpurun_out/r6final2
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_20.log 2>&1 || { tail -5 $O/bench_20.log; exit 1; }
grep '"metric"' $O/bench_20.log | cut -c1-200
OUT=r6final2 DTS=bf16 bash scripts/gpu_r6_j.sh || exit 1
head -14 $O/kernels_bf16.md
