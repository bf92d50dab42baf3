#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/wqprof3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/t -o run -- python3 tools/wq_one.py > $OUT/out.txt 2>&1
echo done
