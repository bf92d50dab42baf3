#!/bin/bash
# d > 8 pass after the scalar LDS-DMA fill loop: timing + bit-identity,
# split sweep at N = M = 1e6.
set -e -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/kde_variants.py 20 262144 default= lds2_1=ABC_KDE_MFMA_LDS2:1 split16=ABC_KDE_MFMA_SPLIT:16 split8=ABC_KDE_MFMA_SPLIT:8 >> $OUT/variants.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_variants.py 20 1000000 default= split16=ABC_KDE_MFMA_SPLIT:16 split8=ABC_KDE_MFMA_SPLIT:8 split64=ABC_KDE_MFMA_SPLIT:64 >> $OUT/variants.txt 2>&1
timeout -k 10 200 python3 -u tools/kde_variants.py 12 262144 default= split16=ABC_KDE_MFMA_SPLIT:16 >> $OUT/variants.txt 2>&1
timeout -k 10 200 python3 -u tools/kde_variants.py 8 1000000 default= split16=ABC_KDE_MFMA_SPLIT:16 >> $OUT/variants.txt 2>&1
echo done
