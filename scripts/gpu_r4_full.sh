#!/bin/bash
# Full check: full GPU test suite, smoke, the 6.7B bench, then a
# kernel trace of the 6.7B step with its timeline (overlap, phases, registers).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels.md > /dev/null
python3 tools/step_timeline.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --md $O/timeline.md
gzip -c "$f" > $O/trace.csv.gz
