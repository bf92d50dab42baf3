#!/bin/bash
# GPU suite with the LDS2 default at d > 8, then the d > 8 variant table.
set -e -o pipefail
OUT=gpurun_out/lds2e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
V="lds2= reg=ABC_KDE_MFMA_LDS2:0"
for d in 20 12 16 24 32; do
timeout -k 10 180 python3 -u tools/kde_variants.py $d 262144 $V > $OUT/d$d.txt 2>&1
done
echo done
