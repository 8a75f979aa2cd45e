#!/bin/bash
# Round 6: paired causal dK/dV grid + 16-byte stores -- numerics, then a
# same-box A/B against the HEAD library: attention rates and the 6.7B step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6ad}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or flash or fa_ or parity" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
H=$(ls tools/fa_lab/_kernels_head.cpython*.so)
for r in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export FLEETX_KERNELS_LIB=$H; else unset FLEETX_KERNELS_LIB; fi
    timeout -k 10 200 python3 tools/bench_attention.py --iters 30 > $O/attn_${v}_$r.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
    timeout -k 10 200 python3 tools/bench_attention.py --h 16 --d 64 --iters 30 >> $O/attn_${v}_$r.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b_${v}_$r.log 2>&1 || { tail -5 $O/b_${v}_$r.log; exit 1; }
    echo $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$r.log) $(grep -o '"final_loss": [0-9.]*' $O/b_${v}_$r.log)
  done
done
unset FLEETX_KERNELS_LIB
for f in $O/attn_*_2.jsonl; do echo $f; cut -c60-230 $f; done
