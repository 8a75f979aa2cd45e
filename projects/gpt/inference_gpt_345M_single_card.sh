#!/bin/bash
# GPT-345M generation through the exported model
# Recipe parity: reference projects/gpt/inference_gpt_345M_single_card.sh
set -e
cd "$(dirname "$0")/../.."
python tasks/gpt/inference.py -c fleetx_amd/configs/nlp/gpt/inference_gpt_345M_single_card.yaml "$@"
