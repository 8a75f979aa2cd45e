#!/bin/bash
# End-of-session check: full GPU suite, smoke, the driver's bench command
# (6.7B, N=1), the 1.3B / 345M benches and ViT-g.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for m in gpt3-1.3B gpt-345M; do
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' $O/bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$m.log) $(grep -o '"mfu": [0-9.]*' $O/bench_$m.log)" | tee -a $O/summary.txt
done
timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/bench_vit_g.log 2>&1 || { tail -20 $O/bench_vit_g.log; exit 1; }
tail -1 $O/bench_vit_g.log | tee -a $O/summary.txt
