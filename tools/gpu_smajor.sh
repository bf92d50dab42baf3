#!/bin/bash
# segment-major default: knob identity, full-size KDE parity, bench
set -e -o pipefail
OUT=gpurun_out/smajor3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "knobs or kde" > $OUT/tests.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
echo done
