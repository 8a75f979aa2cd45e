#!/bin/bash
# Same-box A/B of two builds of the kernel library (ab/old.so vs ab/new.so):
# attention kernels at the GPT-3 6.7B / 345M / ViT-g shapes, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4faab
mkdir -p $O
SO=fleetx_amd/_C/_kernels.cpython-310-x86_64-linux-gnu.so
cp ab/new.so $SO
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or flash or fa_" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for v in old new; do
    cp ab/$v.so $SO
    timeout -k 10 200 python -u tools/bench_attention.py --iters 30 > $O/${v}_${r}_d128.jsonl 2>&1 || exit 1
    timeout -k 10 200 python -u tools/bench_attention.py --iters 30 --h 16 --d 64 > $O/${v}_${r}_d64.jsonl 2>&1 || exit 1
    timeout -k 10 200 python -u tools/bench_attention.py --iters 30 --b 32 --s 257 --h 16 --d 88 > $O/${v}_${r}_d88.jsonl 2>&1 || exit 1
  done
done
cp ab/new.so $SO
python3 - <<'PY'
import json,glob,collections
rows=collections.defaultdict(dict)
for f in sorted(glob.glob('gpurun_out/r4faab/*_d*.jsonl')):
    v,r,d=f.split('/')[-1][:-6].split('_')
    for l in open(f):
        if not l.startswith('{'): continue
        x=json.loads(l); k=(d,x['causal'],x['dropout'])
        rows[k].setdefault(v,[]).append((x['fwd_ms'],x['bwd_ms']))
for k,vv in sorted(rows.items()):
    print(k, {v:(min(a for a,b in t),min(b for a,b in t)) for v,t in vv.items()})
PY
