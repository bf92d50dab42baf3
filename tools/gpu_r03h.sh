#!/bin/bash
# sampled-splitter median / MAD + KDE launch plan at small N: tests + timing
set -e -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_api.py -m gpu -x -v -k "median or mad or adaptive or stat_major or kde or c2 or config" --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
timeout -k 10 200 python3 tools/bench_configs.py --only c2 c1 > $OUT/c2.jsonl 2> $OUT/c2.err
echo done
