#!/bin/bash
# ViT-g/14 knob sweep on one box: AdamW overlap cap, wgrad side stream, dK/dV tile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3vitk
mkdir -p $O
vit() {  # tag, env / -o args...
  local t=$1; shift
  local envs=() args=()
  for a in "$@"; do case $a in FLEETX_*) envs+=("$a");; *) args+=("-o" "$a");; esac; done
  env "${envs[@]}" timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 "${args[@]}" > $O/vit_$t.log 2>&1 || { tail -20 $O/vit_$t.log; exit 1; }
  echo "vit $t $(tail -1 $O/vit_$t.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
}
vit default FLEETX_X=0
vit grid96 Distributed.comm.overlap_optimizer_grid=96
vit grid192 Distributed.comm.overlap_optimizer_grid=192
vit nows Distributed.comm.wgrad_stream=False
vit dkdv32 FLEETX_FA_DKDV=32
vit default2 FLEETX_X=0
