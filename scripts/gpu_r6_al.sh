#!/bin/bash
# Round 6: board power and clocks sampled while the 6.7B / 1.3B / 345M steps
# run (read-only amd-smi queries, back to back, until the bench exits)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6al
mkdir -p $O
rm -f $O/pw_*.jsonl
for spec in "gpt3-6.7B 150" "gpt3-1.3B 600" "gpt-345M 1500"; do
  set -- $spec
  timeout -k 10 400 python3 bench.py --model $1 --steps $2 --warmup 5 > $O/b_$1.log 2>&1 &
  pid=$!
  while kill -0 $pid 2>/dev/null; do
    timeout -k 5 20 amd-smi metric -p -c --json >> $O/pw_$1.jsonl 2>> $O/smi_err.log; echo >> $O/pw_$1.jsonl
  done
  wait $pid || { tail -5 $O/b_$1.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/b_$1.log
done
python3 tools/power_summary.py $O/pw_*.jsonl
