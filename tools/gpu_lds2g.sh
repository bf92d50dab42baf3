#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/lds2g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "knobs or kde_mfma" --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
timeout -k 10 400 python3 -u tools/kde_variants.py 8 1000000 warm= reg1= g1=ABC_KDE_MFMA_LDS2:1 reg2= g2=ABC_KDE_MFMA_LDS2:1 g2ib2=ABC_KDE_MFMA_LDS2:1,ABC_KDE_MFMA_IB:2 > $OUT/kde.txt 2>&1
timeout -k 10 200 python3 -u tools/kde_variants.py 4 100000 warm= reg1= g1=ABC_KDE_MFMA_LDS2:1 reg2= g2=ABC_KDE_MFMA_LDS2:1 >> $OUT/kde.txt 2>&1
echo done
