#!/bin/bash
# Round 5: 64-keys-per-wave dK/dV pass (D = 128): bitwise / reference test, then
# attention timings with it off / on, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ak
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fa_dkdv64_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for r in 1 2; do
  for v in 0 1; do
    FLEETX_FA_DKDV64=$v timeout -k 10 200 python -u tools/bench_attention.py --iters 20 > $O/bench_d128_v${v}_$r.jsonl 2>&1 || { tail -5 $O/bench_d128_v${v}_$r.jsonl; exit 1; }
    echo "dkdv64=$v run $r"; grep -v amdgpu $O/bench_d128_v${v}_$r.jsonl
  done
done
