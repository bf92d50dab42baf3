#!/bin/bash
# Round-2 GPU check: whole -m gpu suite + LocalTransition timings.
set -e -o pipefail
OUT=gpurun_out/r02b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 120 python -u tools/bench_local.py > $OUT/local.txt 2>&1
echo done
