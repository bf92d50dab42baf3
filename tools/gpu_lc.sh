#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/lc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "local_cov" --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
echo done
