#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4fanw
mkdir -p $O
for r in 1 2; do
  for nw in 4 8; do
    FLEETX_FA_FWD_WAVES=$nw timeout -k 10 200 python -u tools/bench_attention.py --iters 30 > $O/nw${nw}_$r.jsonl 2>&1 || exit 1
    FLEETX_FA_FWD_WAVES=$nw timeout -k 10 200 python -u tools/bench_attention.py --iters 30 --h 16 --d 64 > $O/nw${nw}_d64_$r.jsonl 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json,glob,collections
rows=collections.defaultdict(dict)
for f in sorted(glob.glob('gpurun_out/r4fanw/*.jsonl')):
    tag=f.split('/')[-1].split('_')[0]
    for l in open(f):
        if not l.startswith('{'): continue
        x=json.loads(l); k=(x['D'],x['causal'],x['dropout'])
        rows[k].setdefault(tag,[]).append(x['fwd_ms'])
for k,v in sorted(rows.items()): print(k, {t:min(a) for t,a in v.items()})
PY
