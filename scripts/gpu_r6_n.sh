#!/bin/bash
# Round 6: same-box A/B of the small models -- round-start tree (tools/bench_lab/base, its own
# kernel build) vs this tree, and this tree with the vendor TunableOp picks on
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6n
mkdir -p $O
ROOT=$PWD
run() {  # tag dir env -- args
  local tag=$1 dir=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 400 python3 bench.py --model $MODEL --steps 20 --warmup 5 > $O/$tag.log 2>&1) || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }
  echo $tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log) $(grep -o '"mfu": [0-9.]*' $O/$tag.log)
}
for MODEL in gpt-345M gpt3-1.3B; do
  for r in 1 2; do
    run ${MODEL}_base_$r $ROOT/tools/bench_lab/base FLEETX_X=1 || exit 1
    run ${MODEL}_new_$r $ROOT FLEETX_X=1 || exit 1
    run ${MODEL}_newtune_$r $ROOT FLEETX_VENDOR_TUNE=on || exit 1
  done
done
