# GEMM lab sweep on one GPU: tile-group height (FLEETX_GEMM_GM) for the
# hand-scheduled kernel (variant 5) next to hipBLASLt, same process per GM.
set -o pipefail
mkdir -p gpurun_out/g5sweep
for gm in ${GMS:-4 8 16 32}; do
  FLEETX_GEMM_GM=$gm timeout -k 10 200 python tools/bench_gemm.py --iters 30 \
    --only ${CASES:-fwd_x_wT,dgrad_tn_path,wgrad_tn_path,hip_fwd,hip_fwd_gelu,hip_dgrad,hip_wgrad_f32acc} \
    --variants 5 > gpurun_out/g5sweep/gm$gm.log 2>&1 || exit $?
done
