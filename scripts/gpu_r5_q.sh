#!/bin/bash
# Round 5: gemm5 forward (KC x KC) vs data-gradient (KC x MC) PMC at 6.7B shapes;
# 345M with and without the shipped GEMM plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 200 python3 tools/bench_gemm.py --hidden 4096 --only hip_fwd,hip_dgrad,fwd_x_wT,dgrad_tn_path --iters 20 > $O/gemm.jsonl 2>&1 || { tail -5 $O/gemm.jsonl; exit 1; }
cat $O/gemm.jsonl | grep gemm
CTRS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc -o pmc -- python3 tools/bench_gemm.py --hidden 4096 --only hip_fwd,hip_dgrad,fwd_x_wT --iters 3 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
db=$(find $O/pmc -name "*.db" | head -1)
python3 tools/pmc_summary.py "$db" > $O/pmc_summary.txt 2>&1
head -80 $O/pmc_summary.txt
for r in 1 2; do for pl in default none; do
  if [ $pl = none ]; then export FLEETX_GEMM_PLAN=/nonexistent.json; else unset FLEETX_GEMM_PLAN; fi
  timeout -k 10 300 python3 bench.py --model gpt-345M --steps 20 --warmup 5 > $O/b345_${pl}_$r.log 2>&1 || { tail -5 $O/b345_${pl}_$r.log; exit 1; }
  echo 345M plan=$pl $r $(grep -o '"ms_per_step": [0-9.]*' $O/b345_${pl}_$r.log) $(grep -o '"gemm_raced_to_kernel": \[[^]]*\]' $O/b345_${pl}_$r.log)
done; done
