#!/bin/bash
# Column-sum finalize with line-padded tickets + one-pass LayerNorm backward
# with column sums: kernel / fused-norm / parity tests; 345M A/B (LN path,
# workgroups per column reduction); 345M / 1.3B traces; ViT-g bench + trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3cs5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_fused_norm_gpu.py tests/test_model_parity_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
run() {  # tag, env...
  local t=$1; shift
  env "$@" timeout -k 10 400 python bench.py --model gpt-345M --steps 20 --warmup 3 > $O/bench_345M_$t.log 2>&1 || { tail -20 $O/bench_345M_$t.log; exit 1; }
  echo "345M $t $(grep -o '"ms_per_step": [0-9.]*' $O/bench_345M_$t.log)" | tee -a $O/summary.txt
}
run default FLEETX_LN_BWD_FUSED=1
run lnold FLEETX_LN_BWD_FUSED=0
run blocks512 FLEETX_COLSUM_BLOCKS=512
run default2 FLEETX_LN_BWD_FUSED=1
for m in gpt-345M gpt3-1.3B; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$m -o run -- python3 bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  n=$(grep -c adamw_flat "$f"); per=$((n / 5))
  python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_$m.md > /dev/null
  gzip -f "$f"
done
timeout -k 10 500 python tools/bench_vit.py --steps 8 --warmup 3 > $O/bench_vit_g.log 2>&1 || { tail -20 $O/bench_vit_g.log; exit 1; }
tail -1 $O/bench_vit_g.log | tee -a $O/summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_vit -o run -- python3 tools/bench_vit.py --steps 3 --warmup 2 > $O/prof_vit.log 2>&1 || { tail -5 $O/prof_vit.log; exit 1; }
f=$(find $O/prof_vit -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_vit_g.md > /dev/null
gzip -f "$f"
