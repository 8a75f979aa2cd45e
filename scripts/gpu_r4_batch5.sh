#!/bin/bash
# Weight-gradient geometry/split plan + dgrad-only GEMM race: tests, sweep, step A/Bs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_comm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
G=4:1,0:0,8:4,4:4,8:2,4:2,8:1
for h in 1024 1408 2048; do
  timeout -k 10 300 python tools/bench_gemm.py --hidden $h --only hip_wgrad_f32acc --gm 4 --geom $G > $O/geom_h$h.jsonl 2>$O/geom_h$h.err || { tail -5 $O/geom_h$h.err; exit 1; }
done
run() {  # tag, env, args
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("gemm_raced_to_kernel"))')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run s345_$r "FLEETX_GEMM_ROUTE=tune" "--model gpt-345M --steps 20 --warmup 5"
  run s345_oldplan_$r "FLEETX_GEMM_ROUTE=tune FLEETX_GEMM5_F32PLAN=0" "--model gpt-345M --steps 20 --warmup 5"
done
for r in 1 2; do
  run b13_$r "FLEETX_GEMM_ROUTE=tune" "--model gpt3-1.3B --steps 10 --warmup 3"
  run b13_oldplan_$r "FLEETX_GEMM5_F32PLAN=0" "--model gpt3-1.3B --steps 10 --warmup 3"
done
for r in 1 2; do
  run route_$r "FLEETX_GEMM_ROUTE=tune" "--steps 10 --warmup 3"
  run noroute_$r "FLEETX_GEMM_ROUTE=off" "--steps 10 --warmup 3"
done
timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/vit.log 2>&1 || { tail -20 $O/vit.log; exit 1; }
echo "vit $(tail -1 $O/vit.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
FLEETX_GEMM5_F32PLAN=0 timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/vit_old.log 2>&1 || { tail -20 $O/vit_old.log; exit 1; }
echo "vit_oldplan $(tail -1 $O/vit_old.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
