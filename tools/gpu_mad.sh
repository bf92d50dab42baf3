#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/mad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_api.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "median or mad or adaptive or config2" > $OUT/tests.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
echo done
