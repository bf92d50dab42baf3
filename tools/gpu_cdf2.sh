#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/cdf2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $OUT/tr -o run -- python3 tools/probes/cdf_scale.py > $OUT/scale.txt 2>&1
echo done
