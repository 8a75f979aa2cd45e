#!/bin/bash
# Persistent decoder-layer kernel: tests, then generation A/B (same box).
set -o pipefail
O=gpurun_out/r3decl
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --tb=short --timeout 120 --timeout-method thread \
  tests/test_decode_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in 0 1 0 1; do
  FLEETX_DECODE_PERSISTENT=$m timeout -k 10 300 python tools/bench_generation.py --model gpt3-1.3B --batch 1 4 --fused-only > $O/gen_1.3B_$m.jsonl 2>&1 || { tail -5 $O/gen_1.3B_$m.jsonl; exit 1; }
  echo "persistent=$m $(grep ms_per_token $O/gen_1.3B_$m.jsonl | tr '\n' ' ')" | tee -a $O/summary.txt
done
for m in 0 1; do
  FLEETX_DECODE_PERSISTENT=$m timeout -k 10 300 python tools/bench_generation.py --model gpt3-6.7B --batch 1 4 --fused-only > $O/gen_6.7B_$m.jsonl 2>&1 || { tail -5 $O/gen_6.7B_$m.jsonl; exit 1; }
  echo "persistent=$m $(grep ms_per_token $O/gen_6.7B_$m.jsonl | tr '\n' ' ')" | tee -a $O/summary.txt
done
