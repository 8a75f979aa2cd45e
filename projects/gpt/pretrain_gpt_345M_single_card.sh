#!/bin/bash
# GPT-345M pretraining on one MI355X
# Recipe parity: reference projects/gpt/pretrain_gpt_345M_single_card.sh
set -e
cd "$(dirname "$0")/../.."
python tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_345M_single_card.yaml "$@"
