#!/bin/bash
# 6.7B step: bench with optimizer overlap on/off, then a rocprofv3 kernel trace (4 steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2_step
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_overlap_on.log 2>&1 &&
FLEETX_BENCH_OVERRIDES="Distributed.comm.overlap_optimizer=False" \
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_overlap_off.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 4 --warmup 1 > $O/prof.log 2>&1 &&
python3 tools/kernel_summary.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --steps 3 \
  --window embedding_fwd:2:5 --md $O/kernels.md > /dev/null
