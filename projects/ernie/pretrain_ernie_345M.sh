#!/bin/bash
# ERNIE-345M pretraining, one card
# Recipe parity: reference projects/ernie/pretrain_ernie_345M.sh
set -e
cd "$(dirname "$0")/../.."
python tools/train.py -c fleetx_amd/configs/nlp/ernie/pretrain_ernie_345M_single_card.yaml "$@"
