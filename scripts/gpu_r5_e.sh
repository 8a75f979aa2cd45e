#!/bin/bash
# Round 5: co-residency probe -- forward GEMMs on the 128-tile gemm5 geometry
# (2 workgroups per CU at 216 registers per wave: an AdamW wave still fits
# beside them) vs hipBLASLt (512-register waves) in the 6.7B step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
for h in 4096 1024; do
FLEETX_GEMM5_TILE=128 timeout -k 10 300 python3 -u tools/bench_gemm.py --hidden $h --only fwd_x_wT,hip_fwd,hip_fwd_gelu,hip_dgrad --iters 30 > $O/gemm_h${h}_t128.jsonl 2> $O/gemm_h${h}_t128.err || { tail -5 $O/gemm_h${h}_t128.err; exit 1; }
echo "h=$h tile128"; cat $O/gemm_h${h}_t128.jsonl
done
FLEETX_GEMM5_TILE=128 timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py --chunks 66 --paths hip > $O/beside66_t128.jsonl 2> $O/beside66.err || { tail -5 $O/beside66.err; exit 1; }
cat $O/beside66_t128.jsonl
for i in 1 2; do
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_def_$i.log 2>&1 || { tail -5 $O/bench_def_$i.log; exit 1; }
echo def; grep -o '"ms_per_step": [0-9.]*' $O/bench_def_$i.log
FLEETX_GEMM5_TILE=128 FLEETX_GEMM_AUTO=wgrad,fwd timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_fwd128_$i.log 2>&1 || { tail -5 $O/bench_fwd128_$i.log; exit 1; }
echo fwd128; grep -o '"ms_per_step": [0-9.]*' $O/bench_fwd128_$i.log
done
FLEETX_GEMM5_TILE=128 FLEETX_GEMM_AUTO=wgrad,fwd timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); gzip -f "$f"
