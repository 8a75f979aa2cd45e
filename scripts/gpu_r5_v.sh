#!/bin/bash
# Round 5: XCD-rectangle tile mapping for gemm5: bitwise test, GEMM A/B, L2 PMC, step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for xr in 0 1; do
  FLEETX_GEMM_XRECT=$xr timeout -k 10 200 python3 tools/bench_gemm.py --hidden 4096 --only hip_fwd,hip_dgrad,hip_wgrad_f32acc,fwd_x_wT --iters 20 > $O/gemm_x$xr.jsonl 2>&1 || { tail -5 $O/gemm_x$xr.jsonl; exit 1; }
  echo xrect=$xr; grep gemm $O/gemm_x$xr.jsonl
done
CTRS="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
FLEETX_GEMM_XRECT=1 timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc -o pmc -- python3 tools/bench_gemm.py --hidden 4096 --only hip_fwd,hip_dgrad,hip_wgrad_f32acc --iters 3 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
db=$(find $O/pmc -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" > $O/pmc_summary.txt 2>&1
grep -A5 "gemm5" $O/pmc_summary.txt | head -30
for r in 1 2; do for xr in 1 0; do
  FLEETX_GEMM_XRECT=$xr timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 > $O/b67_x${xr}_$r.log 2>&1 || { tail -5 $O/b67_x${xr}_$r.log; exit 1; }
  echo 6.7B xrect=$xr $r $(grep -o '"ms_per_step": [0-9.]*' $O/b67_x${xr}_$r.log)
done; done
