#!/bin/bash
# Round 6: hot-row split of the tied embedding's overlapped update -- graph /
# overlap tests, then a same-box 6.7B A/B (overlap_hot_rows on / off) and the
# small models
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_fp16_gpu.py tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for hr in True False; do
    FLEETX_BENCH_OVERRIDES="Distributed.comm.overlap_hot_rows=$hr" timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_${hr}_$r.log 2>&1 || { tail -5 $O/b_${hr}_$r.log; exit 1; }
    echo hot=$hr $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${hr}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b_${hr}_$r.log)
  done
done
for m in gpt-345M gpt3-1.3B; do
  for hr in True False; do
    FLEETX_BENCH_OVERRIDES="Distributed.comm.overlap_hot_rows=$hr" timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > $O/b_${m}_$hr.log 2>&1 || { tail -5 $O/b_${m}_$hr.log; exit 1; }
    echo $m hot=$hr $(grep -o '"ms_per_step": [0-9.]*' $O/b_${m}_$hr.log) $(grep -o '"final_loss": [0-9.]*' $O/b_${m}_$hr.log)
  done
done
