#!/bin/bash
# Round 5: bf16 vs fp32 gradient storage after dropping the no-collective wire copy
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_grad16_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do for g in bfloat16 float32; do
FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=$g" timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/bench_${g}_$r.log 2>&1 || { tail -5 $O/bench_${g}_$r.log; exit 1; }
echo $g $r $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${g}_$r.log)
done; done
g=bfloat16
FLEETX_BENCH_OVERRIDES="Distributed.comm.grad_dtype=$g" timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$g -o run -- python3 bench.py --steps 3 --warmup 5 > $O/prof_$g.log 2>&1 || { tail -5 $O/prof_$g.log; exit 1; }
f=$(find $O/prof_$g -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --window ce_stats:5:8 --steps 3 --top 25 --md $O/kernels_$g.md > /dev/null
python3 tools/step_timeline.py "$f" --window ce_stats:5:8 --steps 3 --md $O/timeline_$g.md > /dev/null
head -16 $O/kernels_$g.md
gzip -f "$f"
