#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/suite
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
echo done
