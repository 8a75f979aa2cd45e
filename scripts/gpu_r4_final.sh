#!/bin/bash
# End-of-round check: full GPU suite, smoke, 6.7B / 345M / ViT-g benches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_67.log 2>&1 || { tail -20 $O/bench_67.log; exit 1; }
tail -1 $O/bench_67.log
timeout -k 10 300 python bench.py --model gpt-345M --steps 20 --warmup 5 > $O/bench_345.log 2>&1 || { tail -20 $O/bench_345.log; exit 1; }
tail -1 $O/bench_345.log
timeout -k 10 400 python tools/bench_vit.py --steps 10 --warmup 3 > $O/bench_vit.log 2>&1 || { tail -20 $O/bench_vit.log; exit 1; }
tail -1 $O/bench_vit.log
