#!/bin/bash
# rocprofv3 kernel trace of fused batch-1 greedy decode (GPT-3 1.3B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prof_decode}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 tools/bench_generation.py --batch 1 --fused-only --tokens 64 > $OUT/bench.log 2>&1 || { echo "prof failed"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --steps 1 --top 30 --md $OUT/kernels.md > /dev/null 2>&1
head -32 $OUT/kernels.md
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# gaps between consecutive kernels in the last 40% of the trace (steady decode)
tail = rows[int(len(rows) * 0.6):]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail)
span = int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])
print("steady tail: kernels %d, busy %.3f ms, span %.3f ms, busy fraction %.2f" % (len(tail), busy / 1e6, span / 1e6, busy / span))
PY
