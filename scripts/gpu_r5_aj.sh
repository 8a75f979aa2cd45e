#!/bin/bash
# Round 5: 6.7B data-gradient routing A/B in the step, interleaved:
#   def  shipped plan (QKV on gemm5; out / FC1 / FC2 on hipBLASLt + weight transpose)
#   fast plan variant: gemm5 wherever its planned time beats the vendor path at all
#   all  every data gradient on gemm5 (FLEETX_GEMM_AUTO=wgrad,dgrad)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5aj
mkdir -p $O
python3 - <<'PY'
import json
p = json.load(open("fleetx_amd/ops/gemm_plan_gfx950.json"))
for e in p["entries"]:
    if e["kind"] == "dgrad" and e.get("vendor_ms"):
        e["route"] = "kernel" if e["kernel_ms"] < e["vendor_ms"] else "vendor"
json.dump(p, open("/tmp/plan_fast.json", "w"))
PY
v_def=""
v_fast="FLEETX_GEMM_PLAN=/tmp/plan_fast.json"
v_all="FLEETX_GEMM_AUTO=wgrad,dgrad"
for r in 1 2; do
  for v in def fast all; do
    n=v_$v
    env ${!n} timeout -k 10 400 python3 bench.py --steps 10 --warmup 4 > $O/b67_${v}_$r.log 2>&1 || { tail -5 $O/b67_${v}_$r.log; exit 1; }
    echo "6.7B $v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_${v}_$r.log)" | tee -a $O/summary.txt
  done
done
