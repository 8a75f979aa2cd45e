#!/bin/bash
# Imagen super-resolution 512, one card
# Recipe parity: reference projects/imagen/run_super_resolusion_512_single.sh
set -e
cd "$(dirname "$0")/../.."
python tools/train.py -c fleetx_amd/configs/multimodal/imagen/imagen_super_resolusion_512.yaml "$@"
