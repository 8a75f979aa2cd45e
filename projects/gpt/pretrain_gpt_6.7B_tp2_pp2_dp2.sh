#!/bin/bash
# GPT-6.7B TP2 x PP2 x DP2 on 8 MI355X (BASELINE config #3)
# Recipe parity: reference projects/gpt/pretrain_gpt_6.7B_tp2_pp2_dp2.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_hybrid --devices "0,1,2,3,4,5,6,7" --max_restart 3 tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_6.7B_tp2_pp2_dp2.yaml "$@"
