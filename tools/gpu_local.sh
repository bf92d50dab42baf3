#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/local
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_api.py tests/test_gpu_distributed.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "local" > $OUT/tests.txt 2>&1
timeout -k 10 120 python -u tools/bench_local.py > $OUT/bench_local.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_configs.py --only c4 > $OUT/c4.jsonl 2> $OUT/c4.err
echo done
