#!/bin/bash
# Checkpoint: whole -m gpu suite on the working tree, then configs 1 and 2
set -e -o pipefail
OUT=gpurun_out/chk
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 300 python3 -u tools/bench_configs.py --only c1 c2 c4 > $OUT/configs.jsonl 2> $OUT/configs.err
echo done
