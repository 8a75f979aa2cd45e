#!/bin/bash
# Fused LM-head cross-entropy: GPU tests (single rank, TP2, TP2+SP vs the plain
# head), then time / peak memory A/B on 345M and 6.7B (same box).
set -o pipefail
O=gpurun_out/r3head
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --tb=short --timeout 300 --timeout-method thread \
  tests/test_multirank_gpu.py -k "fused_lm_head" > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for m in gpt-345M gpt3-6.7B; do
  st=20; [ $m = gpt3-6.7B ] && st=10
  for f in False True; do
    FLEETX_BENCH_OVERRIDES="Model.fused_lm_head_ce=$f" timeout -k 10 400 python bench.py --model $m --steps $st --warmup 3 > $O/bench_${m}_$f.log 2>&1 || { tail -20 $O/bench_${m}_$f.log; exit 1; }
    echo "$m fused=$f $(grep -o '"value": [0-9.]*' $O/bench_${m}_$f.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${m}_$f.log) $(grep -o '"final_loss": [0-9.]*' $O/bench_${m}_$f.log) $(grep -o '"peak_mem_gb": [0-9.]*' $O/bench_${m}_$f.log)" | tee -a $O/summary.txt
  done
done
