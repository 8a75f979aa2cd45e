#!/bin/bash
# Round 6 end, continued: FA lab tests, default-config bench (driver K/W), 6.7B kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6final2
mkdir -p $O
FLEETX_KERNELS_LIB=$(ls tools/fa_lab/_kernels.cpython*.so) timeout -k 10 300 python -u -m pytest tools/fa_lab/test_fa_wave64_lab.py -x -q --timeout 120 --timeout-method thread > $O/fa_lab.log 2>&1 || { tail -20 $O/fa_lab.log; exit 1; }
tail -1 $O/fa_lab.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_20_$r.log 2>&1 || { tail -5 $O/bench_20_$r.log; exit 1; }
grep '"metric"' $O/bench_20_$r.log | cut -c1-200
done
OUT=r6final2 DTS=bf16 bash scripts/gpu_r6_j.sh || exit 1
head -14 $O/kernels_bf16.md
