#!/bin/bash
# Round 5: L2 hit / miss of gemm5 vs hipBLASLt at the 6.7B layer shapes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
CTRS="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc -o pmc -- python3 tools/bench_gemm.py --hidden 4096 --only hip_fwd,hip_dgrad,fwd_x_wT,hip_wgrad_f32acc --iters 3 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
db=$(find $O/pmc -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" > $O/pmc_summary.txt 2>&1
grep -A6 "gemm5\|Cijk" $O/pmc_summary.txt | head -60
CTRS2="GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $CTRS2 -d $O/pmc2 -o pmc -- python3 tools/bench_gemm.py --hidden 4096 --only hip_fwd,fwd_x_wT --iters 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
db=$(find $O/pmc2 -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" > $O/pmc2_summary.txt 2>&1
grep -A6 "gemm5\|Cijk" $O/pmc2_summary.txt | head -40
