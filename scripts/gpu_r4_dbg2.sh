#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4dbg
mkdir -p $O
timeout -k 10 200 python -u scripts/debug_overlap_adamw.py > $O/dbg2.log 2>&1; echo "rc=$?"; tail -30 $O/dbg2.log
