#!/bin/bash
# GPU suite, kernel table and end-to-end configs after the async population
# offload and the pairwise Philox normals.
set -e -o pipefail
OUT=gpurun_out/r02e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
timeout -k 10 400 python3 -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
echo done
