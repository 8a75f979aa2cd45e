#!/bin/bash
# Round 6: side-stream (overlapped AdamW) HIP priority A/B on the 6.7B step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6r
mkdir -p $O
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for r in 1 2; do for p in 0 -5 5; do
  FLEETX_SIDE_PRIORITY=$p timeout -k 10 300 python3 bench.py --steps 15 --warmup 5 > $O/b_p${p}_$r.log 2>&1 || { tail -5 $O/b_p${p}_$r.log; exit 1; }
  echo prio=$p $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_p${p}_$r.log)
done; done
