#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4defer
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_kernels_gpu.py -x -q -k "graph or overlapped" --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E|Error" $O/pytest.log | head -20; exit 1; }
run() {
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(tail -1 $O/$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["mfu"], d["final_loss"])')" | tee -a $O/summary.txt
}
for r in 1 2; do
  run s345_defer_$r "X=1" "--model gpt-345M --steps 20 --warmup 5"
  run s345_serial_$r "FLEETX_BENCH_OVERRIDES=Distributed.comm.overlap_optimizer=False" "--model gpt-345M --steps 20 --warmup 5"
done
