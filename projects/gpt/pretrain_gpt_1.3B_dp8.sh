#!/bin/bash
# GPT-1.3B data parallel on 8 MI355X
# Recipe parity: reference projects/gpt/pretrain_gpt_1.3B_dp8.sh
set -e
cd "$(dirname "$0")/../.."
log_dir=log_dp8; rm -rf $log_dir
python -m fleetx_amd.launch --log_dir $log_dir --devices "0,1,2,3,4,5,6,7" tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_1.3B_dp8.yaml "$@"
