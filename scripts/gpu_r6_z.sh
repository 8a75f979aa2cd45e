#!/bin/bash
# Round 6: FA forward stamps, shipped tile body vs the full (unmasked) body on the causal grid
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6z}
mkdir -p $O
for v in "" _fa_exp_nomask; do
  L=$(ls tools/fa_lab/_kernels${v}.cpython*.so)
  FLEETX_KERNELS_LIB=$L timeout -k 10 200 python3 tools/fa_lab/stamp_fwd.py > $O/stamps$v.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  head -1 $O/stamps$v.jsonl | cut -c1-700
done
