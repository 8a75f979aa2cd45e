#!/bin/bash
# Round 5: paired causal attention forward; AdamW G16 load order; grad16 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_grad16_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do for pr in 0 1; do
FLEETX_FA_PAIR=$pr timeout -k 10 120 python3 tools/bench_attention.py --iters 50 > $O/attn_pair${pr}_$r.jsonl 2>&1 || { tail -5 $O/attn_pair${pr}_$r.jsonl; exit 1; }
echo pair=$pr; grep '"causal": true' $O/attn_pair${pr}_$r.jsonl
done; done
for r in 1 2; do for g in bfloat16 float32; do
FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=$g" timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/bench_${g}_$r.log 2>&1 || { tail -5 $O/bench_${g}_$r.log; exit 1; }
echo $g $r $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${g}_$r.log)
done; done
