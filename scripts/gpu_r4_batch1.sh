#!/bin/bash
# Round 4 batch: multirank + w^T cache tests, gm sweep, AdamW placement / w^T cache step A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b1
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_multirank_gpu.py tests/test_wt_cache_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
OUT=r4b1/gm bash scripts/gpu_r4_gm.sh > /dev/null || exit 1
run() {  # tag, overrides
  FLEETX_BENCH_OVERRIDES="$2" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run wt_$r ""
  run nowt_$r "Distributed.comm.cache_transposed_weights=False"
  run cu32_$r "Distributed.comm.overlap_optimizer_cus=32"
  run cu64_$r "Distributed.comm.overlap_optimizer_cus=64"
done
run serial "Distributed.comm.overlap_optimizer=False"
