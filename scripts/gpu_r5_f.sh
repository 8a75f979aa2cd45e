#!/bin/bash
# Round 5: persistent gemm5 with exact MAIN wait (buffer-store epilogue) -- tests,
# bench, step A/B; AdamW rate vs workgroups
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_gemm.log 2>&1 || { tail -30 $O/test_gemm.log; exit 1; }
tail -2 $O/test_gemm.log
timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py --grid-sweep 32,64,96,128,192,256 --wide 1 > $O/adamw_grid_wide.jsonl 2>&1 || { tail -5 $O/adamw_grid_wide.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py --grid-sweep 64,128,256,512 --wide 0 > $O/adamw_grid.jsonl 2>&1 || { tail -5 $O/adamw_grid.jsonl; exit 1; }
cat $O/adamw_grid_wide.jsonl $O/adamw_grid.jsonl | grep adamw
for p in 1 0; do
FLEETX_GEMM5_PERSIST=$p timeout -k 10 300 python3 -u tools/bench_gemm.py --hidden 4096 --only fwd_x_wT,hip_fwd,hip_fwd_gelu,hip_dgrad,hip_dgrad_dgelu --iters 30 > $O/gemm_p$p.jsonl 2> $O/gemm_p$p.err || { tail -5 $O/gemm_p$p.err; exit 1; }
echo "persist=$p"; cat $O/gemm_p$p.jsonl
done
for i in 1 2; do
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_def_$i.log 2>&1 || { tail -5 $O/bench_def_$i.log; exit 1; }
echo def; grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9a-zA-Z.]*' $O/bench_def_$i.log
FLEETX_GEMM_AUTO=wgrad,fwd timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_fwd_$i.log 2>&1 || { tail -5 $O/bench_fwd_$i.log; exit 1; }
echo fwd; grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9a-zA-Z.]*' $O/bench_fwd_$i.log
done
