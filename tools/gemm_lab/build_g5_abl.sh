#!/bin/bash
# gemm5 ablation lab binaries: bin/g5_<abl> with the K-loop regenerated
# without one instruction class (tools/gen_gemm_asm.py FX_GEN_ABL).
set -e
cd "$(dirname "$0")"
mkdir -p bin gen
for abl in ${G5ABLS:-none novm nodma nobar nolds nodma,nolds}; do
  tag=${abl//,/_}
  if [ "$abl" = none ]; then a=""; else a=$abl; fi
  FX_GEN_ABL=$a FX_GEN_OUT=gen/g5_$tag.inc python ../gen_gemm_asm.py
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DFX_GEMM5_INC="\"$(pwd)/gen/g5_$tag.inc\"" \
    -o bin/g5_$tag gemm_lab.cpp gemm_legacy.hip ../../csrc/kernels/gemm5.hip &
done
wait
ls -la bin
