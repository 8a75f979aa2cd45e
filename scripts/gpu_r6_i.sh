#!/bin/bash
# Round 6: sumsq_16 test + fp16/grad16 tests; fp16 O2 6.7B step (graph) vs bf16, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_grad16_gpu.py tests/test_fp16_gpu.py tests/test_gemm_gpu.py > $O/t.log 2>&1 || { echo FAIL; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  echo $name $(grep -o '"value": [0-9.]*' $O/$name.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log) $(grep -o '"final_loss": [0-9.]*' $O/$name.log) $(grep -o '"hip_graph": [a-z]*' $O/$name.log)
}
run bf16 FLEETX_X=1
run fp16 FLEETX_BENCH_OVERRIDES=Engine.mix_precision.dtype=float16
run fp16_fusednorm "FLEETX_BENCH_OVERRIDES=Engine.mix_precision.dtype=float16;Distributed.comm.fused_grad_norm=True"
