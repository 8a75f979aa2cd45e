#!/bin/bash
# GPT-6.7B sharding (ZeRO) over 2x8 MI355X; run on both nodes with NODE_RANK=0/1 and MASTER=ip:port
# Recipe parity: reference projects/gpt/pretrain_gpt_6.7B_sharding16.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_sharding16 --devices "0,1,2,3,4,5,6,7" --nnodes 2 --node_rank ${NODE_RANK:-0} --master ${MASTER:-127.0.0.1:29500} tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_6.7B_sharding16.yaml "$@"
