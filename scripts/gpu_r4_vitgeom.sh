#!/bin/bash
# ViT-g weight-gradient shapes (16448 tokens): geometry / split sweep.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4vitgeom
mkdir -p $O
G=4:1,0:0,8:1,8:2,8:3,8:4,8:5,8:6,8:7,8:8,4:2,4:3
timeout -k 10 400 python tools/bench_gemm.py --tokens 16448 --hidden 1408 --ffn 6144 --only hip_wgrad_f32acc --gm 4 --geom $G --iters 10 > $O/vit.jsonl 2>$O/vit.err || { tail -5 $O/vit.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4vitgeom/vit.jsonl'):
    d=json.loads(l)
    ks=[k for k in d if k.startswith('hip_wgrad')]
    print(d['gemm'], d['N'], d['K'], ' '.join('%s=%.0f'%(k.split('_g')[-1],d[k]) for k in ks))
PY
