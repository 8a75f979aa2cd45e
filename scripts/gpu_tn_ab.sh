#!/bin/bash
# A/B of the TN transposes (wgrad / dgrad) on the small models, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for m in ${MODELS:-gpt-345M gpt3-1.3B}; do
  for combo in "1 1" "0 1" "1 0" "0 0" "1 1"; do
    set -- $combo
    r=$(FLEETX_WGRAD_TN=$1 FLEETX_DGRAD_TN=$2 timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null | grep '^{') || { echo "fail $m $combo"; exit 1; }
    echo "$m WGRAD_TN=$1 DGRAD_TN=$2 $(echo $r | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["mfu"])')"
  done
done
