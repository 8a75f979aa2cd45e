#!/bin/bash
# Fused gradient norm: kernel + engine tests, then the 6.7B step A/B (same box).
set -o pipefail
O=gpurun_out/r3fnorm
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_fused_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for cfg in "fused:" "plain:Distributed.comm.fused_grad_norm=False" "fused2:"; do
  tag=${cfg%%:*}; ov=${cfg#*:}
  FLEETX_BENCH_OVERRIDES="$ov" timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/bench_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $O/bench_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.log) $(grep -o '"final_loss": [0-9.]*' $O/bench_$tag.log)" | tee -a $O/summary.txt
done
bash scripts/gpu_r3_small_prof.sh
