#!/bin/bash
# AdamW kernel variants (non-temporal mode x block shape) at full grid and the 128 cap.
# (ran with profiles/r4_adamw/variants.patch applied; the --variants sweep was not kept)
set -o pipefail
O=gpurun_out/r4adamw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_optim_semantics.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_optim.py --n 1e9 --iters 10 --variants > $O/variants.jsonl 2>&1 || { tail -20 $O/variants.jsonl; exit 1; }
grep -v amdgpu $O/variants.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d.get('kernel'), d.get('grid'), d.get('nontemporal'), d.get('block'), d.get('float4_per_thread'), d['ms'], d['TB_s'])"
