#!/bin/bash
# LocalTransition density on the f32 MFMA: tests (incl. C4 full size), timing
set -e -o pipefail
OUT=gpurun_out/lm
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "local" --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_api.py tests/test_gpu_distributed.py -m gpu -x -v -s -k "local or c4" --timeout 240 --timeout-method thread > $OUT/tests2.txt 2>&1
timeout -k 10 200 python3 -u tools/bench_local.py > $OUT/bench_local.txt 2>&1
timeout -k 10 200 python3 tools/bench_configs.py --only c4 > $OUT/c4.jsonl 2>&1
echo done
