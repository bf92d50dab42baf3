#!/bin/bash
# engine sync consolidation + strided stat-major views: tests, C2/C4 timers,
# d = 4 KDE launch knobs at C2's size
set -e -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_api.py -m gpu -x -v -k "stat_major or decide or guard or pnorm or median or std or c2 or config or adaptive or singlecore or record" --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
timeout -k 10 200 python3 tools/bench_configs.py --only c2 c2 c4 > $OUT/c2.jsonl 2> $OUT/c2.err
timeout -k 10 200 python3 -u tools/kde_variants.py 4 100000 default= split16=ABC_KDE_MFMA_SPLIT:16 split32=ABC_KDE_MFMA_SPLIT:32 ib1=ABC_KDE_MFMA_IB:1 ib2=ABC_KDE_MFMA_IB:2 pipe0=ABC_KDE_MFMA_PIPE:0 > $OUT/kde4.txt 2>&1
echo done
