#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/lds2f
mkdir -p $OUT
export TMPDIR=/tmp
V="lds2= fold=ABC_KDE_MFMA_LDS2:1,ABC_KDE_MFMA_FOLD:1 ilv=ABC_KDE_MFMA_LDS2:2 ilv_ib1=ABC_KDE_MFMA_LDS2:2,ABC_KDE_MFMA_IB:1 ilv_s16=ABC_KDE_MFMA_LDS2:2,ABC_KDE_MFMA_SPLIT:16"
for d in 20 12 24 32; do
timeout -k 10 200 python3 -u tools/kde_variants.py $d 262144 $V > $OUT/d$d.txt 2>&1
done
echo done
