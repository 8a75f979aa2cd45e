#!/bin/bash
# Builds the GEMM lab binaries into tools/gemm_lab/bin:
#   gemm_lab_abl{0..3}: csrc/kernels/gemm.hip (+ gemm5.hip), normal and ablation builds
#   gemm_lab_stamp:     s_memtime stamps (FX_GEMM_STAMP=1)
# ABLS="0" limits the set (e.g. only the normal build).
set -e
cd "$(dirname "$0")"
mkdir -p bin
for abl in ${ABLS:-0 1 2 3}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DFX_GEMM_ABL=$abl $EXTRA \
    -o bin/gemm_lab_abl$abl gemm_lab.cpp gemm_legacy.hip ../../csrc/kernels/gemm5.hip &
done
if [ -z "$ABLS" ]; then
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DFX_GEMM_STAMP=1 \
  -o bin/gemm_lab_stamp gemm_lab.cpp gemm_legacy.hip ../../csrc/kernels/gemm5.hip &
fi
wait
ls -la bin
