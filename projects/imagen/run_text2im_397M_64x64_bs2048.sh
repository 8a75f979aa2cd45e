#!/bin/bash
# Imagen 397M text-to-image 64x64, dp8
# Recipe parity: reference projects/imagen/run_text2im_397M_64x64_bs2048.sh
set -e
cd "$(dirname "$0")/../.."
python -m fleetx_amd.launch --log_dir log_imagen --devices "0,1,2,3,4,5,6,7" tools/train.py -c fleetx_amd/configs/multimodal/imagen/imagen_397M_text2im_64x64.yaml -o Distributed.dp_degree=8 -o Data.Train.loader.num_workers=8 -o Engine.num_train_epochs=68 "$@"
