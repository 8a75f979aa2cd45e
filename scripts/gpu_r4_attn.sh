#!/bin/bash
# Attention: timings + one PMC pass (causal vs non-causal, fwd/bwd kernels).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4attn}
mkdir -p $O
timeout -k 10 200 python -u tools/bench_attention.py --iters 20 > $O/bench_d128.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_attention.py --iters 20 --h 16 --d 64 > $O/bench_d64.jsonl 2>&1 || exit 1
CTRS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc -o pmc -- python3 tools/bench_attention.py --iters 3 > $O/pmc.log 2>&1 || exit 1
db=$(find $O/pmc -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" --filter fa_ > $O/pmc_summary.txt 2>&1
grep -v amdgpu $O/bench_d128.jsonl $O/bench_d64.jsonl
