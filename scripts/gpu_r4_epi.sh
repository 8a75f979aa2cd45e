#!/bin/bash
# hipBLASLt GELU epilogues vs plain GEMMs at the 6.7B / 1.3B / 345M MLP shapes.
set -o pipefail
O=gpurun_out/r4epi
mkdir -p $O
timeout -k 10 120 tools/bin/hipblaslt_epi_probe 8192 4096 16384 > $O/p67.txt 2>&1 || { cat $O/p67.txt; exit 1; }
timeout -k 10 120 tools/bin/hipblaslt_epi_probe 8192 2048 8192 > $O/p13.txt 2>&1 || { cat $O/p13.txt; exit 1; }
timeout -k 10 120 tools/bin/hipblaslt_epi_probe 8192 1024 4096 > $O/p345.txt 2>&1 || { cat $O/p345.txt; exit 1; }
cat $O/p67.txt; grep case $O/p13.txt $O/p345.txt
