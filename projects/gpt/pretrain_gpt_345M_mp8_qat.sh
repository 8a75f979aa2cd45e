#!/bin/bash
# GPT-345M tensor parallel 8 with QAT fake-quant
# Recipe parity: reference projects/gpt/pretrain_gpt_345M_mp8_qat.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_qat --devices "0,1,2,3,4,5,6,7" tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_345M_mp8_qat.yaml "$@"
