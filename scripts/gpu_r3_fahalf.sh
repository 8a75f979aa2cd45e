#!/bin/bash
# Flash-attention forward / dQ skip fully masked 32-key halves (causal diagonal,
# S = 257 tail): attention tests, then isolated A/B (FLEETX_FA_HALF_SKIP) on
# the 6.7B / 345M / ViT-g shapes and the 6.7B / ViT-g steps.
set -o pipefail
export TMPDIR=/tmp
O=${FAH_OUT:-gpurun_out/r3fah}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py -k "flash" > $O/pytest.log 2>&1 && FLEETX_FA_DQ_HALF_SKIP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py -k "flash" >> $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for hs in 1 0 1; do
  FLEETX_FA_DQ_HALF_SKIP=$hs FLEETX_FA_HALF_SKIP=$hs timeout -k 10 200 python tools/bench_attention.py > $O/attn128_$hs.jsonl 2>/dev/null || exit 1
  FLEETX_FA_DQ_HALF_SKIP=$hs FLEETX_FA_HALF_SKIP=$hs timeout -k 10 200 python tools/bench_attention.py --h 16 --d 64 > $O/attn64_$hs.jsonl 2>/dev/null || exit 1
  FLEETX_FA_DQ_HALF_SKIP=$hs FLEETX_FA_HALF_SKIP=$hs timeout -k 10 200 python tools/bench_vit_attention.py > $O/attnvit_$hs.jsonl 2>/dev/null || exit 1
  echo "half_skip=$hs"; grep -h '"causal": true, "dropout": 0.1\|fwd_ms' $O/attn128_$hs.jsonl $O/attn64_$hs.jsonl $O/attnvit_$hs.jsonl | grep -o '"D": [0-9]*\|"causal": [a-z]*\|"dropout": [0-9.]*\|"fwd_ms": [0-9.]*' | paste -sd' ' | tee -a $O/summary.txt
done
for hs in 1 0; do
  FLEETX_FA_DQ_HALF_SKIP=$hs FLEETX_FA_HALF_SKIP=$hs timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench67_$hs.log 2>&1 || exit 1
  echo "6.7B half_skip=$hs $(grep -o '"ms_per_step": [0-9.]*' $O/bench67_$hs.log)" | tee -a $O/summary.txt
  FLEETX_FA_DQ_HALF_SKIP=$hs FLEETX_FA_HALF_SKIP=$hs timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/vit_$hs.log 2>&1 || exit 1
  echo "vit half_skip=$hs $(tail -1 $O/vit_$hs.log | grep -o '"value": [0-9.]*')" | tee -a $O/summary.txt
done
