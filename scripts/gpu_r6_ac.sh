#!/bin/bash
# Round 6: per-wave stamps of the attention dK/dV pass (lab build), causal vs full
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6ac}
mkdir -p $O
L=$(ls tools/fa_lab/_kernels.cpython*.so)
FLEETX_KERNELS_LIB=$L timeout -k 10 200 python3 tools/fa_lab/stamp_bwd.py > $O/stamps_bwd.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
python3 -c "
import json
for l in open('$O/stamps_bwd.jsonl'):
    d=json.loads(l); kb=d.pop('by_kblock'); print(d)
    for r in kb: print('  ', r)
"
