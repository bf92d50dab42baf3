#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/ilv
mkdir -p $OUT
export TMPDIR=/tmp
ABC_KDE_MFMA_LDS2=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 400 --timeout-method thread -k "d20 or 20" > $OUT/fullsize.txt 2>&1 || true
cp gpurun_out/kde_fullsize_parity.json $OUT/ 2>/dev/null || true
echo done
