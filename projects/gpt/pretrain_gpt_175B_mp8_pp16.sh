#!/bin/bash
# GPT-175B mp8 x pp16 over 16 nodes (NODE_RANK / MASTER per node)
# Recipe parity: reference projects/gpt/pretrain_gpt_175B_mp8_pp16.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_hybrid --devices "0,1,2,3,4,5,6,7" --nnodes 16 --node_rank ${NODE_RANK:-0} --master ${MASTER:-127.0.0.1:29500} tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_175B_mp8_pp16.yaml "$@"
