#!/bin/bash
set -o pipefail
bash scripts/gpu_r3_declayer.sh; r1=$?
echo "declayer rc=$r1"
[ $r1 -eq 0 ] || [ $r1 -eq 1 ] || exit $r1
bash scripts/gpu_r3_multirank.sh || exit 1
bash scripts/gpu_r3_dkdv.sh
