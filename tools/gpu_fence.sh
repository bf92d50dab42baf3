#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/fence
mkdir -p $OUT
export TMPDIR=/tmp
V="default= fence=ABC_KDE_MFMA_FENCE:1 default2= fence2=ABC_KDE_MFMA_FENCE:1"
timeout -k 10 300 python3 -u tools/kde_variants.py 8 1000000 $V > $OUT/d8.txt 2>&1
timeout -k 10 200 python3 -u tools/kde_variants.py 4 100000 $V > $OUT/d4.txt 2>&1
echo done
