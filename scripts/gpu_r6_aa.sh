#!/bin/bash
# Round 6: 16-byte O stores in the attention forward -- numerics, stamps, rates
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6aa}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or flash or fa_" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$(ls tools/fa_lab/_kernels.cpython*.so)
FLEETX_KERNELS_LIB=$L timeout -k 10 200 python3 tools/fa_lab/stamp_fwd.py > $O/stamps.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
cut -c1-420 $O/stamps.jsonl
for r in 1 2; do
timeout -k 10 200 python3 tools/bench_attention.py --iters 30 > $O/attn_$r.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
timeout -k 10 200 python3 tools/bench_attention.py --h 16 --d 64 --iters 30 >> $O/attn_$r.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
cat $O/attn_*.jsonl | cut -c1-230
