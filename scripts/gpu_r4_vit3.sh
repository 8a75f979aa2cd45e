#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4vit3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 > $O/vit_$r.log 2>&1 || { tail -20 $O/vit_$r.log; exit 1; }
  echo "vit_$r $(tail -1 $O/vit_$r.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
done
