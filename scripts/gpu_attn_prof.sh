#!/bin/bash
# Kernel-only attention timings: rocprofv3 kernel stats of tools/bench_attention.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/attn}; mkdir -p $OUT
export TMPDIR=/tmp

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_attention.py $ATTN_ARGS > $OUT/bench.log 2>&1
rc=$?
cat $OUT/bench.log | grep '^{'
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "fa_" in n or "flash" in n:
        print("%-90s calls=%5s avg_us=%8.1f" % (n[:90], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
exit $rc
