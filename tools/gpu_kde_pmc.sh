#!/bin/bash
# PMC pass over the MFMA KDE at d=20 for the register and the DMA variants.
set -e -o pipefail
OUT=gpurun_out/kde_pmc
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/base20 -o run -- python3 tools/kde_one.py 262144 20 > $OUT/base20.out 2>&1
ABC_KDE_MFMA_DMA=1 timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/dma20 -o run -- python3 tools/kde_one.py 262144 20 > $OUT/dma20.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/base8 -o run -- python3 tools/kde_one.py 262144 8 > $OUT/base8.out 2>&1
echo done
