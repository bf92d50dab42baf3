#!/bin/bash
# KDE + LocalTransition GPU tests after the d > 8 split default and the
# diagnostics cleanup, the C4 full-size test, a PMC pass over the new d > 8
# kernel, and a bench line with the extended CPU baseline.
set -e -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_api.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
cp gpurun_out/kde_fullsize_parity.json $OUT/
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/pmc20a -o run -- python3 tools/kde_one.py 262144 20 > $OUT/pmc20a.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C2 -T -f csv -d $OUT/pmc20b -o run -- python3 tools/kde_one.py 262144 20 > $OUT/pmc20b.out 2>&1
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
echo done
