#!/bin/bash
# gm autotune: GEMM numerics, then 6.7B step with tuning on vs off (2 rounds).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
run() {  # tag, env
  env $2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run tune_$r "FLEETX_GEMM_TUNE=1"
  run notune_$r "FLEETX_GEMM_TUNE=0"
  run tune_dgrad_$r "FLEETX_GEMM_AUTO=wgrad,dgrad"
done
