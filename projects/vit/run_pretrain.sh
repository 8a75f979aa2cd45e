#!/bin/bash
# ViT-B/16 ImageNet pretraining, dp8 bf16
# Recipe parity: reference projects/vit/run_pretrain.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_vit --devices "0,1,2,3,4,5,6,7" tools/train.py -c fleetx_amd/configs/vis/vit/ViT_base_patch16_224_pt_in1k_2n16c_dp_fp16o2.yaml "$@"
