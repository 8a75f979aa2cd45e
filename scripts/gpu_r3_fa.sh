#!/bin/bash
# Persistent flash-attention forward: tests, kernel A/B, 6.7B / 1.3B step A/B.
set -o pipefail
O=gpurun_out/r3fa
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py -k "flash_attention" > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in 0 1; do
  FLEETX_FA_PERSISTENT=$m timeout -k 10 200 python tools/bench_attention.py > $O/attn_$m.jsonl 2>&1 || { tail -5 $O/attn_$m.jsonl; exit 1; }
  FLEETX_FA_PERSISTENT=$m timeout -k 10 200 python tools/bench_attention.py --d 64 --h 16 > $O/attn_d64_$m.jsonl 2>&1 || { tail -5 $O/attn_d64_$m.jsonl; exit 1; }
done
grep -h '"causal": true' $O/attn_*.jsonl
for m in 1 0 1; do
  for model in gpt3-6.7B gpt3-1.3B; do
    st=20; [ $model = gpt3-6.7B ] && st=10
    FLEETX_FA_PERSISTENT=$m timeout -k 10 400 python bench.py --model $model --steps $st --warmup 3 > $O/bench_${model}_$m.log 2>&1 || { tail -20 $O/bench_${model}_$m.log; exit 1; }
    echo "$model persistent=$m $(grep -o '"value": [0-9.]*' $O/bench_${model}_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${model}_$m.log)" | tee -a $O/summary.txt
  done
done
