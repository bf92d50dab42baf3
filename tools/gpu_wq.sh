#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/wq3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py tests/test_gpu_api.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "quantile or epsilon or two_ranks or rccl or config" > $OUT/tests.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
echo done
