#!/bin/bash
# Round 5: runner-up rectangle cuts in the tile-order codes: tests, plan regeneration, step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5y
mkdir -p $O
mkdir -p gpurun_ab
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python3 -u tools/gemm_plan.py --out $O/gemm_plan_gfx950.json > $O/plan.jsonl 2> $O/plan.err || { tail -5 $O/plan.err; exit 1; }
tail -1 $O/plan.err
for r in 1 2; do for pl in new cur; do
  if [ $pl = new ]; then PF=$O/gemm_plan_gfx950.json; else PF=fleetx_amd/ops/gemm_plan_gfx950.json; fi
  FLEETX_GEMM_PLAN=$PF timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_${pl}_$r.log 2>&1 || { tail -5 $O/b67_${pl}_$r.log; exit 1; }
  echo 6.7B plan=$pl $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_${pl}_$r.log)
done; done
for r in 1 2; do for pl in new cur; do
  if [ $pl = new ]; then PF=$O/gemm_plan_gfx950.json; else PF=fleetx_amd/ops/gemm_plan_gfx950.json; fi
  FLEETX_GEMM_PLAN=$PF timeout -k 10 300 python3 tools/bench_vit.py > $O/vit_${pl}_$r.log 2>&1 || { tail -5 $O/vit_${pl}_$r.log; exit 1; }
  echo vit plan=$pl $r $(grep -o '"value": [0-9.]*' $O/vit_${pl}_$r.log | tail -1)
done; done
