#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/pk2
mkdir -p $OUT
export TMPDIR=/tmp
V="lds2= pk=ABC_KDE_MFMA_PK:1 lds2b= pkb=ABC_KDE_MFMA_PK:1"
for d in 20 12 24; do
timeout -k 10 200 python3 -u tools/kde_variants.py $d 262144 $V > $OUT/d$d.txt 2>&1
done
echo done
