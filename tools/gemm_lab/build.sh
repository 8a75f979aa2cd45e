#!/bin/bash
# Builds the GEMM lab binaries (normal + ablations) into tools/gemm_lab/bin.
set -e
cd "$(dirname "$0")"
mkdir -p bin
for abl in 0 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DFX_GEMM_ABL=$abl $EXTRA \
    -o bin/gemm_lab_abl$abl gemm_lab.cpp ../../csrc/kernels/gemm.hip &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DFX_GEMM_STAMP=1 \
  -o bin/gemm_lab_stamp gemm_lab.cpp ../../csrc/kernels/gemm.hip &
wait
ls -la bin
