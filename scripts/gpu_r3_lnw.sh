#!/bin/bash
# One-pass LayerNorm backward with column sums at h 2048 / 4096 (2 / 4 waves
# per row): kernel / fused-norm / parity tests, then 1.3B and 6.7B A/B against
# the two-pass path, and a 6.7B kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3lnw
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_fused_norm_gpu.py tests/test_model_parity_gpu.py tests/test_graph_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
gpt() {  # model, tag, steps, env...
  local m=$1 t=$2 n=$3; shift 3
  env "$@" timeout -k 10 400 python bench.py --model $m --steps $n --warmup 3 > $O/gpt_${m}_$t.log 2>&1 || { tail -20 $O/gpt_${m}_$t.log; exit 1; }
  echo "$m $t $(grep -o '"ms_per_step": [0-9.]*' $O/gpt_${m}_$t.log)" | tee -a $O/summary.txt
}
gpt gpt3-1.3B fused 20 FLEETX_LN_BWD_FUSED=1
gpt gpt3-1.3B twopass 20 FLEETX_LN_BWD_FUSED=0
gpt gpt3-6.7B fused 10 FLEETX_LN_BWD_FUSED=1
gpt gpt3-6.7B twopass 10 FLEETX_LN_BWD_FUSED=0
gpt gpt3-6.7B fused2 10 FLEETX_LN_BWD_FUSED=1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_6.7B.md > /dev/null
gzip -f "$f"
