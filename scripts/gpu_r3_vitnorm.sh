#!/bin/bash
# ViT linears feed the fused gradient norm from the wgrad epilogue: fused-norm
# / parity tests, ViT-g bench and a kernel trace (sumsq_chunks per step).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3vitn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_fused_norm_gpu.py tests/test_model_parity_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python tools/bench_vit.py --steps 8 --warmup 3 > $O/bench_vit_g.log 2>&1 || { tail -20 $O/bench_vit_g.log; exit 1; }
tail -1 $O/bench_vit_g.log | tee -a $O/summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_vit -o run -- python3 tools/bench_vit.py --steps 3 --warmup 2 > $O/prof_vit.log 2>&1 || { tail -5 $O/prof_vit.log; exit 1; }
f=$(find $O/prof_vit -name "*kernel_trace.csv" | head -1)
n=$(grep -c adamw_flat "$f"); per=$((n / 5))
python3 tools/kernel_summary.py "$f" --window adamw_flat:$((2 * per)):$((5 * per)) --steps 3 --top 40 --md $O/kernels_vit_g.md > /dev/null
gzip -f "$f"
