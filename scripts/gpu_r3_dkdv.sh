#!/bin/bash
# dK/dV with 64-query tiles and V in registers (D <= 96): tests, kernel and
# 345M step A/B (same box).
set -o pipefail
O=gpurun_out/r3dkdv
mkdir -p $O
FLEETX_FA_DKDV=64 timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py -k "flash_attention" > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in 32 64 32 64; do
  FLEETX_FA_DKDV=$m timeout -k 10 200 python tools/bench_attention.py --d 64 --h 16 > $O/attn_d64_$m.jsonl 2>&1 || { tail -5 $O/attn_d64_$m.jsonl; exit 1; }
  echo "dkdv=$m $(grep '"causal": true, "dropout": 0.1' $O/attn_d64_$m.jsonl)" | tee -a $O/summary.txt
done
for m in 32 64 32 64; do
  FLEETX_FA_DKDV=$m timeout -k 10 300 python bench.py --model gpt-345M --steps 20 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  echo "345M dkdv=$m $(grep -o '"value": [0-9.]*' $O/bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log)" | tee -a $O/summary.txt
done
