#!/bin/bash
# Last check of HEAD: full GPU suite (default paths), the dQ half-skip tests,
# then the flash-attention A/B with the dQ skip on / off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3last
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
FAH_OUT=gpurun_out/r3fah2 bash scripts/gpu_r3_fahalf.sh
