#!/bin/bash
# Stored-dS attention backward: numerics, then old (recompute) vs new attention bench.
# (ran with profiles/r4_ds/stored_ds.patch applied; FLEETX_FA_BWD_DS was not kept)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ds
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash or attn" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E|assert|Error" $O/pytest.log | head -30; exit 1; }
for f in 1 0; do
  FLEETX_FA_BWD_DS=$f timeout -k 10 200 python -u tools/bench_attention.py --iters 30 > $O/attn_d128_ds$f.jsonl 2>&1 || exit 1
  FLEETX_FA_BWD_DS=$f timeout -k 10 200 python -u tools/bench_attention.py --iters 30 --h 16 --d 64 > $O/attn_d64_ds$f.jsonl 2>&1 || exit 1
  FLEETX_FA_BWD_DS=$f timeout -k 10 200 python -u tools/bench_attention.py --iters 30 --b 64 --s 257 --h 16 --d 88 > $O/attn_d88_ds$f.jsonl 2>&1 || exit 1
done
for f in $O/attn_*.jsonl; do echo "== $f"; grep -v amdgpu $f; done
