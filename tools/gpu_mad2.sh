#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/mad2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_api.py -m gpu -x -q -k "median or mad or adaptive" --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
timeout -k 10 120 python3 tools/mad_one.py > $OUT/mad.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/st -o run -- python3 tools/mad_one.py > $OUT/mad_prof.txt 2>&1
echo done
