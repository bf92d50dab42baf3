#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py tests/test_gpu_api.py -m gpu -x -v -s -k "quantile or two_ranks_equal or epsilon or config" --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1
cat > /tmp/ab.sh <<'EOS'
for i in 1 2 3; do
python3 -u tools/kde_variants.py 4 100000 default= old=ABC_KDE_MFMA_PIPE:1,ABC_KDE_MFMA_SPLIT:64
done
EOS
timeout -k 10 300 bash /tmp/ab.sh > $OUT/kde_ab.txt 2>&1
echo done
