#!/bin/bash
# GPT-345M zero-shot text generation
# Recipe parity: reference projects/gpt/generation_gpt_345M_single_card.sh
set -e
cd "$(dirname "$0")/../.."
python tasks/gpt/generation.py -c fleetx_amd/configs/nlp/gpt/generation_gpt_345M_single_card.yaml "$@"
