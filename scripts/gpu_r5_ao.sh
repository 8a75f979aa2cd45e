#!/bin/bash
# Round 5: transposed 16-bit weight gradient for wide shapes (FC2): test,
# microbench, 6.7B step A/B interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ao
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "transposed or tile_order or xcd" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 200 python -u tools/bench_wgrad_t.py > $O/bench_wgrad_t.jsonl 2>&1 || { tail -5 $O/bench_wgrad_t.jsonl; exit 1; }
cat $O/bench_wgrad_t.jsonl
for r in 1 2; do
  for v in 0 1; do
    FLEETX_GEMM_WGRAD_T=$v timeout -k 10 400 python3 bench.py --steps 10 --warmup 4 > $O/b67_t${v}_$r.log 2>&1 || { tail -5 $O/b67_t${v}_$r.log; exit 1; }
    echo "6.7B wgrad_t=$v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_t${v}_$r.log)" | tee -a $O/summary.txt
  done
done
