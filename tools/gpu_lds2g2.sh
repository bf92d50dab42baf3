#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/lds2g2
mkdir -p $OUT
export TMPDIR=/tmp
G2=ABC_KDE_MFMA_LDS2:1,ABC_KDE_MFMA_IB:2
G1=ABC_KDE_MFMA_LDS2:1,ABC_KDE_MFMA_IB:1
timeout -k 10 600 python3 -u tools/kde_variants.py 8 1000000 warm= reg1= g2a=$G2 g1a=$G1 reg2= g2b=$G2 g1b=$G1 reg3= g2c=$G2 g2s16=$G2,ABC_KDE_MFMA_SPLIT:16 g2s64=$G2,ABC_KDE_MFMA_SPLIT:64 > $OUT/kde.txt 2>&1
echo done
