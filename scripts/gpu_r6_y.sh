#!/bin/bash
# Round 6: per-wave stamps of the flash-attention forward (lab build), causal vs full
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6y}
mkdir -p $O
L=$(ls tools/fa_lab/_kernels.cpython*.so)
FLEETX_KERNELS_LIB=$L timeout -k 10 200 python3 tools/fa_lab/stamp_fwd.py > $O/stamps.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
FLEETX_KERNELS_LIB=$L timeout -k 10 200 python3 tools/fa_lab/stamp_fwd.py --h 16 --d 64 > $O/stamps_d64.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
cut -c1-900 $O/stamps.jsonl
