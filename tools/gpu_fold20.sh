#!/bin/bash
# Folded accumulation at d = 12 / 16 / 20 (KL 6 / 7 / 9): launch-shape sweep,
# rows against the fp64 pass and against the split-order DMA variant.
set -e -o pipefail
OUT=gpurun_out/fold20
mkdir -p $OUT
export TMPDIR=/tmp
V="default= pipe=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SCHED:0 sched=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SCHED:1 ib1=ABC_KDE_MFMA_IB:1 ib1pipe=ABC_KDE_MFMA_IB:1,ABC_KDE_MFMA_PIPE:1 split_dma=ABC_KDE_MFMA_DMA:1"
timeout -k 10 180 python3 -u tools/kde_variants.py 20 262144 $V > $OUT/d20.txt 2>&1
timeout -k 10 180 python3 -u tools/kde_variants.py 16 262144 $V > $OUT/d16.txt 2>&1
timeout -k 10 180 python3 -u tools/kde_variants.py 12 262144 $V > $OUT/d12.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_variants.py 20 1000000 default= split_dma=ABC_KDE_MFMA_DMA:1 > $OUT/d20_1e6.txt 2>&1
echo done
