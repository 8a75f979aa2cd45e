#!/bin/bash
# LayerNorm returning its input as the residual alias (no separate gradient
# add): model parity / graph / fp16 / multirank tests, then same-box A/B on
# 345M, 6.7B and ViT-g.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3keep
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --tb=short --timeout 300 --timeout-method thread \
  tests/test_model_parity_gpu.py tests/test_graph_gpu.py tests/test_fp16_gpu.py tests/test_kernels_gpu.py \
  tests/test_multirank_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
gpt() {  # model, tag, steps, env...
  local m=$1 t=$2 n=$3; shift 3
  env "$@" timeout -k 10 400 python bench.py --model $m --steps $n --warmup 3 > $O/gpt_${m}_$t.log 2>&1 || { tail -20 $O/gpt_${m}_$t.log; exit 1; }
  echo "$m $t $(grep -o '"ms_per_step": [0-9.]*' $O/gpt_${m}_$t.log) $(grep -o '"final_loss": [0-9.]*' $O/gpt_${m}_$t.log)" | tee -a $O/summary.txt
}
vit() {  # tag, env...
  local t=$1; shift
  env "$@" timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/vit_$t.log 2>&1 || { tail -20 $O/vit_$t.log; exit 1; }
  echo "vit $t $(tail -1 $O/vit_$t.log | grep -o '"value": [0-9.]*\|"final_loss": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
}
gpt gpt-345M keep 20 FLEETX_LN_KEEP_INPUT=1
gpt gpt-345M plain 20 FLEETX_LN_KEEP_INPUT=0
gpt gpt3-6.7B keep 10 FLEETX_LN_KEEP_INPUT=1
gpt gpt3-6.7B plain 10 FLEETX_LN_KEEP_INPUT=0
vit keep FLEETX_LN_KEEP_INPUT=1
vit plain FLEETX_LN_KEEP_INPUT=0
