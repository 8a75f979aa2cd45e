#!/bin/bash
# FA transposed reads from asm (no vmcnt(0) on the prefetch) + per-shape GEMM
# routing: kernel tests, attention bench, wgrad geometry sweep, step A/Bs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_attention.py --iters 20 > $O/attn_d128.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_attention.py --iters 20 --h 16 --d 64 > $O/attn_d64.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_attention.py --iters 20 --b 32 --s 257 --h 16 --d 88 > $O/attn_d88.jsonl 2>&1 || exit 1
grep -v amdgpu $O/attn_*.jsonl
G=0:0,4:1,4:2,4:3,4:4,8:1,8:2,8:4
for h in 1024 1408 2048; do
  v=""; [ $h = 1024 ] && v="--vocab 50304"
  timeout -k 10 300 python tools/bench_gemm.py --hidden $h $v --only hip_wgrad_f32acc,wgrad_tn_path --gm 4 --geom $G > $O/geom_h$h.jsonl 2>$O/geom_h$h.err || { tail -5 $O/geom_h$h.err; exit 1; }
done
run() {  # tag, env, args
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run route_$r "FLEETX_GEMM_ROUTE=tune" "--steps 10 --warmup 3"
  run noroute_$r "FLEETX_GEMM_ROUTE=off" "--steps 10 --warmup 3"
done
for r in 1 2; do
  run s345_route_$r "FLEETX_GEMM_ROUTE=tune" "--model gpt-345M --steps 20 --warmup 5"
  run s345_noroute_$r "FLEETX_GEMM_ROUTE=off" "--model gpt-345M --steps 20 --warmup 5"
done
