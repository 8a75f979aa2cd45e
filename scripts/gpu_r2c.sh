#!/bin/bash
# Round-2 re-entry check: GPU tests, smoke, 6.7B bench, ViT-g engine steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_check.sh || exit $?
timeout -k 10 240 python -u scripts/debug_vit_step.py fleetx_amd/configs/vis/vit/ViT_g_patch14_224_synthetic_dp8.yaml > gpurun_out/vit_g.log 2>&1
rc=$?; tail -8 gpurun_out/vit_g.log; exit $rc
