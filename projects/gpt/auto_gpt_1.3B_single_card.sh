#!/bin/bash
# GPT-1.3B semi-auto parallel, one card
# Recipe parity: reference projects/gpt/auto_gpt_1.3B_single_card.sh
set -e
cd "$(dirname "$0")/../.."
python tools/auto.py -c fleetx_amd/configs/nlp/gpt/auto/pretrain_gpt_1.3B_single_card.yaml "$@"
