#!/bin/bash
# Kernel trace of config 2 (N = 1e5, d = 4, AdaptivePNorm MAD) end to end
set -e -o pipefail
OUT=gpurun_out/c2trace
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -T -f csv -d $OUT/tr -o run -- python3 tools/bench_configs.py --only c2 > $OUT/c2.jsonl 2> $OUT/c2.err
echo done
