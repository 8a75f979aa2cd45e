#!/bin/bash
# Round 5: persistent gemm5 (16-bit outputs) -- tests, beside-AdamW probe, 6.7B step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_gemm.log 2>&1 || { tail -30 $O/test_gemm.log; exit 1; }
tail -2 $O/test_gemm.log
timeout -k 10 300 python3 -u tools/bench_gemm_beside_adamw.py --chunks 66 > $O/beside66.jsonl 2> $O/beside66.err || { tail -5 $O/beside66.err; exit 1; }
cat $O/beside66.jsonl
for i in 1 2; do
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_def_$i.log 2>&1 || { tail -5 $O/bench_def_$i.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench_def_$i.log
FLEETX_GEMM_AUTO=wgrad,fwd timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 5 > $O/bench_fwd_$i.log 2>&1 || { tail -5 $O/bench_fwd_$i.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench_fwd_$i.log
done
