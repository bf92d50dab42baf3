#!/bin/bash
# The whole -m gpu suite + smoke on HEAD (no bench / profile)
set -e -o pipefail
OUT=gpurun_out/final_suite
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
echo done
