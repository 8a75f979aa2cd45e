#!/bin/bash
# GPT-345M offline evaluation (WikiText PPL / LAMBADA with -o Offline_Eval.cloze_eval=True)
# Recipe parity: reference projects/gpt/evaluate_gpt_345M_single_card.sh
set -e
cd "$(dirname "$0")/../.."
python tools/eval.py -c fleetx_amd/configs/nlp/gpt/eval_gpt_345M_single_card.yaml "$@"
