#!/bin/bash
# fused simulate + distance: tests, the distributed / bench paths, the bench
set -e -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -m gpu -x -v -k "fused or decide or stat_major or median or kde or guard or pnorm or rank or bench" --timeout 280 --timeout-method thread > $OUT/tests.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 200 python3 -u tools/kde_variants.py 4 100000 default= > $OUT/kde4.txt 2>&1
echo done
