#!/bin/bash
# One GPU validation pass (run on the MI355X box via gpurun): kernel/unit GPU
# tests, the attention micro-benchmark, the headline bench and a rocprofv3
# kernel-stats profile of the bench.  Every GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-5}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_attention.py > $OUT/attn.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps $STEPS --warmup 2 > $OUT/bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- \
    python bench.py --steps 3 --warmup 1 > $OUT/prof.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/attn.log 2>/dev/null; tail -2 $OUT/bench.log 2>/dev/null
exit $rc
