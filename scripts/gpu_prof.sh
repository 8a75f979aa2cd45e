#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py $BENCH_ARGS > gpurun_out/prof/bench_prof.log 2>&1
rc=$?
tail -3 gpurun_out/prof/bench_prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
