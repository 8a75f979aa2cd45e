#!/bin/bash
# Round 5: packed fp32 master (bf16 hi + 16-bit lo): tests + step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_packed_master_gpu.py tests/test_grad16_gpu.py tests/test_optim_semantics.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for pk in True False; do
  FLEETX_BENCH_OVERRIDES="Optimizer.packed_master=$pk" timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_pk${pk}_$r.log 2>&1 || { tail -5 $O/b67_pk${pk}_$r.log; exit 1; }
  echo 6.7B packed=$pk $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_pk${pk}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b67_pk${pk}_$r.log) $(grep -o '"peak_mem_gb": [0-9.]*' $O/b67_pk${pk}_$r.log)
done; done
for r in 1 2; do for pk in True False; do
  FLEETX_BENCH_OVERRIDES="Optimizer.packed_master=$pk" timeout -k 10 300 python3 bench.py --model gpt-345M --steps 20 --warmup 5 > $O/b345_pk${pk}_$r.log 2>&1 || { tail -5 $O/b345_pk${pk}_$r.log; exit 1; }
  echo 345M packed=$pk $r $(grep -o '"ms_per_step": [0-9.]*' $O/b345_pk${pk}_$r.log)
done; done
