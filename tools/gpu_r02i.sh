#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/r02i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
cp gpurun_out/kde_fullsize_parity.json $OUT/
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
timeout -k 10 400 python3 -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
echo done
