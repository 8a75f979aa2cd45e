#!/bin/bash
# GPT-6.7B semi-auto parallel sharding16 (2 nodes)
# Recipe parity: reference projects/gpt/auto_gpt_6.7B_sharding16.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_auto --devices "0,1,2,3,4,5,6,7" --nnodes 2 --node_rank ${NODE_RANK:-0} --master ${MASTER:-127.0.0.1:29500} tools/auto.py -c fleetx_amd/configs/nlp/gpt/auto/pretrain_gpt_6.7B_sharding16.yaml "$@"
