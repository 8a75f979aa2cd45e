#!/bin/bash
# Round 5: one-wave-per-SIMD dK/dV and dQ passes (D = 128): bitwise / reference test, then
# attention timings with it off / on, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ak
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fa_wave64_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for r in 1 2; do
  for v in 00 10 01 11; do
    FLEETX_FA_DKDV64=${v:0:1} FLEETX_FA_DQ64=${v:1:1} timeout -k 10 200 python -u tools/bench_attention.py --iters 20 > $O/bench_d128_v${v}_$r.jsonl 2>&1 || { tail -5 $O/bench_d128_v${v}_$r.jsonl; exit 1; }
    echo "dkdv64,dq64=$v run $r"; grep -v amdgpu $O/bench_d128_v${v}_$r.jsonl
  done
done
