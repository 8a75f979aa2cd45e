#!/bin/bash
# GPT-345M export for the inference engine
# Recipe parity: reference projects/gpt/export_gpt_345M_single_card.sh
set -e
cd "$(dirname "$0")/../.."
python tools/export.py -c fleetx_amd/configs/nlp/gpt/generation_gpt_345M_single_card.yaml "$@"
