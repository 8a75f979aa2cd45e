#!/bin/bash
# Round 6: fused gradient norm back on under the fp16 loss scaler -- fp16 tests,
# then a same-box fp16 6.7B A/B (fused norm on / off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp16_gpu.py tests/test_fused_norm_gpu.py tests/test_grad16_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for fn in True False; do
    FLEETX_BENCH_OVERRIDES="Engine.mix_precision.dtype=float16;Distributed.comm.fused_grad_norm=$fn" timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_${fn}_$r.log 2>&1 || { tail -5 $O/b_${fn}_$r.log; exit 1; }
    echo fused=$fn $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${fn}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b_${fn}_$r.log) $(grep -o '"dtype": "[a-z0-9]*"' $O/b_${fn}_$r.log)
  done
done
