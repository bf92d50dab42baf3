#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/kde_variants.py 4 100000 warm= old1=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64 new1= old2=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64 new2= old3=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64 new3= > $OUT/kde_ab.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_variants.py 8 100000 warm= old1=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64 new1= old2=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64 new2= >> $OUT/kde_ab.txt 2>&1
echo done
