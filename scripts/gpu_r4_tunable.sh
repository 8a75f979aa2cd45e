#!/bin/bash
# PyTorch TunableOp over the hipBLASLt / rocBLAS GEMMs (forward + vendor data
# gradients): tune once into a results file, then run with tuning off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4tun
mkdir -p $O
export PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tunableop_6.7B%d.csv
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/base.log 2>&1 || { tail -5 $O/base.log; exit 1; }
echo "base $(tail -1 $O/base.log | cut -c1-200)"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
echo "tune $(tail -1 $O/tune.log | cut -c1-200)"
ls -la $O
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/tuned.log 2>&1 || { tail -5 $O/tuned.log; exit 1; }
echo "tuned $(tail -1 $O/tuned.log | cut -c1-200)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/base2.log 2>&1 || { tail -5 $O/base2.log; exit 1; }
echo "base2 $(tail -1 $O/base2.log | cut -c1-200)"
