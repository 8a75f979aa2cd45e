#!/bin/bash
# 6.7B 1-GPU bench with different FLEETX_GEMM_AUTO kind sets (which GEMMs use the HIP kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for kinds in ${KINDS:-none fwd_act dgrad_act wgrad fwd_act,dgrad_act}; do
  echo "== FLEETX_GEMM_AUTO=$kinds"
  FLEETX_GEMM=auto FLEETX_GEMM_AUTO=$kinds timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_auto_$kinds.log 2>&1
  rc=$?
  tail -1 gpurun_out/bench_auto_$kinds.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_auto_$kinds.log; exit $rc; fi
done
