#!/bin/bash
# gemm5 schedule variants: bin/g5v_<tag>, each with the K-loop regenerated
# under the given generator knobs, e.g.
#   VARIANTS="s1g4:FX_GEN_STAGGER=1,FX_GEN_DMA_GAP=4 s0g3:FX_GEN_STAGGER=0,FX_GEN_DMA_GAP=3"
set -e
cd "$(dirname "$0")"
mkdir -p bin gen
for v in $VARIANTS; do
  tag=${v%%:*}
  envs=${v#*:}
  env ${envs//,/ } FX_GEN_OUT=gen/g5v_$tag.inc python ../gen_gemm_asm.py
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../csrc/kernels -DFX_GEMM5_INC="\"$(pwd)/gen/g5v_$tag.inc\"" \
    -o bin/g5v_$tag gemm_lab.cpp gemm_legacy.hip ../../csrc/kernels/gemm5.hip &
done
wait
