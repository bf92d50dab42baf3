#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/knn
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 120 python -u tools/bench_local.py > $OUT/rows8.txt 2>&1
ABC_KNN_ROWS=16 timeout -k 10 120 python -u tools/bench_local.py > $OUT/rows16.txt 2>&1
ABC_KNN_ROWS=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "knn" > $OUT/tests16.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
echo done
