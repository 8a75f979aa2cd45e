#!/bin/bash
# gemm5 split-K (quarter-full last wave rule, wider combine): GEMM / parity
# tests; ViT-g split on / off; 345M / 1.3B with the default routing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3sk2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_fused_norm_gpu.py tests/test_model_parity_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
vit() {  # tag, env...
  local t=$1; shift
  env "$@" timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/vit_$t.log 2>&1 || { tail -20 $O/vit_$t.log; exit 1; }
  echo "vit $t $(tail -1 $O/vit_$t.log | grep -o '"value": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')" | tee -a $O/summary.txt
}
gpt() {  # model, tag, env...
  local m=$1 t=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 3 > $O/gpt_${m}_$t.log 2>&1 || { tail -20 $O/gpt_${m}_$t.log; exit 1; }
  echo "$m $t $(grep -o '"ms_per_step": [0-9.]*' $O/gpt_${m}_$t.log)" | tee -a $O/summary.txt
}
vit default FLEETX_GEMM5_SPLITK=1
vit nosplit FLEETX_GEMM5_SPLITK=0 FLEETX_GEMM_WGRAD_MIN_TILES=192
vit default2 FLEETX_GEMM5_SPLITK=1
gpt gpt-345M default FLEETX_GEMM5_SPLITK=1
gpt gpt-345M nosplit FLEETX_GEMM5_SPLITK=0 FLEETX_GEMM_WGRAD_MIN_TILES=192
gpt gpt3-1.3B default FLEETX_GEMM5_SPLITK=1
gpt gpt3-1.3B nosplit FLEETX_GEMM5_SPLITK=0 FLEETX_GEMM_WGRAD_MIN_TILES=192
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_vit -o run -- python3 tools/bench_vit.py --steps 3 --warmup 2 > $O/prof_vit.log 2>&1 || { tail -5 $O/prof_vit.log; exit 1; }
f=$(find $O/prof_vit -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_vit_g.md > /dev/null
gzip -f "$f"
