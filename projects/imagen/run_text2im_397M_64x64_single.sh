#!/bin/bash
# Imagen 397M text-to-image 64x64, one card
# Recipe parity: reference projects/imagen/run_text2im_397M_64x64_single.sh
set -e
cd "$(dirname "$0")/../.."
python tools/train.py -c fleetx_amd/configs/multimodal/imagen/imagen_397M_text2im_64x64.yaml "$@"
