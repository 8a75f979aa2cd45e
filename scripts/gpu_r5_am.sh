#!/bin/bash
# Round 5: D = 128 dK/dV with V in registers (2 waves per SIMD): test + timings
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fa_wave64_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for r in 1 2; do
  for v in 0 1; do
    FLEETX_FA_DKDV_VREG=$v timeout -k 10 200 python -u tools/bench_attention.py --iters 20 > $O/bench_d128_vreg${v}_$r.jsonl 2>&1 || { tail -5 $O/bench_d128_vreg${v}_$r.jsonl; exit 1; }
    echo "vreg=$v run $r $(grep -o '"bwd_ms": [0-9.]*' $O/bench_d128_vreg${v}_$r.jsonl | awk '{printf "%s ", $2}')"
  done
done
