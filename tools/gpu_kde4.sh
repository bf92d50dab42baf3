#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/kde4
mkdir -p $OUT
export TMPDIR=/tmp
for d in 4 3 2 1 6; do
timeout -k 10 200 python3 -u tools/kde_variants.py $d 100000 default= pipe0=ABC_KDE_MFMA_PIPE:0 pipe0_ib2=ABC_KDE_MFMA_PIPE:0,ABC_KDE_MFMA_IB:2 pipe0_ib1=ABC_KDE_MFMA_PIPE:0,ABC_KDE_MFMA_IB:1 pipe0_s32=ABC_KDE_MFMA_PIPE:0,ABC_KDE_MFMA_SPLIT:32 pipe0_ib2_s32=ABC_KDE_MFMA_PIPE:0,ABC_KDE_MFMA_IB:2,ABC_KDE_MFMA_SPLIT:32 >> $OUT/kde.txt 2>&1
done
timeout -k 10 200 python3 -u tools/kde_variants.py 4 1000000 default= pipe0=ABC_KDE_MFMA_PIPE:0 pipe0_ib2=ABC_KDE_MFMA_PIPE:0,ABC_KDE_MFMA_IB:2 >> $OUT/kde.txt 2>&1
timeout -k 10 200 python3 -u tools/kde_variants.py 8 1000000 default= pipe0=ABC_KDE_MFMA_PIPE:0 >> $OUT/kde.txt 2>&1
echo done
