#!/bin/bash
# GPT-1.3B semi-auto parallel dp8
# Recipe parity: reference projects/gpt/auto_gpt_1.3B_dp8.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_auto --devices "0,1,2,3,4,5,6,7" tools/auto.py -c fleetx_amd/configs/nlp/gpt/auto/pretrain_gpt_1.3B_dp8.yaml "$@"
