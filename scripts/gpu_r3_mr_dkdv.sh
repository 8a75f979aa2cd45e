#!/bin/bash
set -o pipefail
bash scripts/gpu_r3_multirank.sh || exit 1
bash scripts/gpu_r3_dkdv.sh
