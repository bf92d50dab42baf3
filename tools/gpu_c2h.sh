#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/c2h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/c2_hostprof.py > $OUT/prof.txt 2> $OUT/prof.err
timeout -k 10 200 python3 -u tools/kde_variants.py 4 100000 default= > $OUT/kde.txt 2>&1
timeout -k 10 200 python3 tools/bench_configs.py --only c2 c1 > $OUT/c2.jsonl 2> $OUT/c2.err
echo done
