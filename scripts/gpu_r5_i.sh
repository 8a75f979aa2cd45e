#!/bin/bash
# Round 5: full GPU suite (plan, grad16, PP overlap), 6.7B step A/B of bf16 gradient storage
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "per-tensor worst|passed|failed" $O/pytest_gpu.log | tail -40
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_g16_$i.log 2>&1 || { tail -5 $O/bench_g16_$i.log; exit 1; }
echo g16; grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9a-zA-Z.]*\|"peak_mem_gb": [0-9.]*\|"gemm_raced_to_kernel": [^]]*' $O/bench_g16_$i.log
FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=float32" timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_g32_$i.log 2>&1 || { tail -5 $O/bench_g32_$i.log; exit 1; }
echo g32; grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9a-zA-Z.]*\|"peak_mem_gb": [0-9.]*' $O/bench_g32_$i.log
done
