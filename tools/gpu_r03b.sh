#!/bin/bash
# d > 8 interleaved split pass: bit-identity against the compiler-scheduled
# split pass and the register kernel, timing at d = 12 / 20 / 24; the d = 8
# default unchanged; the KDE GPU tests.
set -e -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
V="default= lds2_1=ABC_KDE_MFMA_LDS2:1 lds2_0=ABC_KDE_MFMA_LDS2:0 fold=ABC_KDE_MFMA_FOLD:1 split16=ABC_KDE_MFMA_SPLIT:16 ib1=ABC_KDE_MFMA_IB:1"
for d in 20 12 24; do
  timeout -k 10 200 python3 -u tools/kde_variants.py $d 262144 $V >> $OUT/variants.txt 2>&1
done
timeout -k 10 200 python3 -u tools/kde_variants.py 20 1000000 default= fold=ABC_KDE_MFMA_FOLD:1 >> $OUT/variants.txt 2>&1
timeout -k 10 200 python3 -u tools/kde_variants.py 8 1000000 default= pipe0=ABC_KDE_MFMA_PIPE:0 >> $OUT/variants.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -x -v -s -k "kde" --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
cp gpurun_out/kde_fullsize_parity.json $OUT/
echo done
