#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/c2t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_configs.py --only c2 c2 c4 > $OUT/c2.jsonl 2> $OUT/c2.err
echo done
