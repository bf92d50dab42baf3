#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -s -k "quantile" --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
cat > /tmp/ab.sh <<'EOS'
for i in 1 2 3; do
python3 -u tools/kde_variants.py 4 100000 default= old=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64
done
EOS
timeout -k 10 300 bash /tmp/ab.sh > $OUT/kde_ab.txt 2>&1
echo done
