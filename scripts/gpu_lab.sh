#!/bin/bash
# GEMM lab runs: variants x ablations, then one PMC pass on the normal build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=tools/gemm_lab/bin
for abl in ${ABLS:-0 1 2}; do
  for v in ${VARS:-0 1}; do
    echo "abl=$abl variant=$v"
    timeout -k 10 120 $B/gemm_lab_abl$abl $v 10 || exit 1
  done
done 2>&1 | tee gpurun_out/lab.log
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
  cd $GRAFT_REPO_ROOT
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --stats -d gpurun_out/pmc -o pmc -- $B/gemm_lab_abl0 0 3 > gpurun_out/pmc.log 2>&1
  echo "pmc rc=$?"
fi
