#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/slp2
mkdir -p $OUT
export TMPDIR=/tmp
L=pyabc_amd/_lib/noslp/libabc_hip.so
timeout -k 10 300 python3 -u tools/kde_ab.py $L 8 1000000 nosched=ABC_KDE_MFMA_SCHED:0 default= nosched_s16=ABC_KDE_MFMA_SCHED:0,ABC_KDE_MFMA_SPLIT:16 > $OUT/d8_noslp.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_variants.py 8 1000000 default= nosched=ABC_KDE_MFMA_SCHED:0 > $OUT/d8_slp.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_ab.py $L 20 262144 default= > $OUT/d20_noslp.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_variants.py 20 262144 default= > $OUT/d20_slp.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_ab.py $L 4 100000 default= nosched=ABC_KDE_MFMA_SCHED:0 > $OUT/d4_noslp.txt 2>&1
timeout -k 10 300 python3 -u tools/kde_variants.py 4 100000 default= nosched=ABC_KDE_MFMA_SCHED:0 > $OUT/d4_slp.txt 2>&1
echo done
