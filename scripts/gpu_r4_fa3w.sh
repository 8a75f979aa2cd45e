#!/bin/bash
# 3-wave workgroups for 96-wide attention tiles (ViT-g): tests, attention bench, ViT step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4fa3w
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash or attn" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 200 python -u tools/bench_attention.py --iters 30 --b 64 --s 257 --h 16 --d 88 > $O/attn_d88.jsonl 2>&1 || exit 1
grep -v amdgpu $O/attn_d88.jsonl
for r in 1 2; do
  timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 > $O/vit_$r.log 2>&1 || { tail -20 $O/vit_$r.log; exit 1; }
  echo "vit_$r $(tail -1 $O/vit_$r.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
done
