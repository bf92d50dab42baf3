#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/r02f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 400 python3 -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
echo done
