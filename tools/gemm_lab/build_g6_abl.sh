#!/bin/bash
# VGPR-staged gemm5 K-loop ablations: bin/g6_<abl> (FX_GEN_ABL classes removed;
# timing only, results wrong).  ABLS="none novm ..." limits the set.
set -e
cd "$(dirname "$0")"
mkdir -p bin gen
for abl in ${ABLS:-none novm nodma nowr nolds nobar}; do
  a=$abl; [ "$a" = none ] && a=""
  FX_GEN_ABL=$a FX_GEN_OUT=gen/g6_$abl.inc python ../gen_gemm_asm.py
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DFX_GEMM5_INC="\"$(pwd)/gen/g6_$abl.inc\"" \
    -o bin/g6_$abl gemm_lab.cpp ../../csrc/kernels/gemm.hip ../../csrc/kernels/gemm5.hip &
done
wait
