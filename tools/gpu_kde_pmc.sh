#!/bin/bash
# PMC passes over the MFMA KDE at d = 20 (register / LDS2 / LDS2 folded):
# matrix-pipe busy, VALU / MFMA issue, wave cycles and the effective clock.
set -e -o pipefail
OUT=gpurun_out/kde_pmc20
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/base -o run -- python3 tools/kde_one.py 262144 20 > $OUT/base.out 2>&1
ABC_KDE_MFMA_LDS2=1 ABC_KDE_MFMA_SPLIT=16 timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/lds2 -o run -- python3 tools/kde_one.py 262144 20 > $OUT/lds2.out 2>&1
ABC_KDE_MFMA_LDS2=1 ABC_KDE_MFMA_FOLD=1 ABC_KDE_MFMA_SPLIT=16 timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/fold -o run -- python3 tools/kde_one.py 262144 20 > $OUT/fold.out 2>&1
ABC_KDE_MFMA_LDS2=1 ABC_KDE_MFMA_SPLIT=16 timeout -s KILL 120 rocprofv3 --pmc $C2 -T -f csv -d $OUT/lds2b -o run -- python3 tools/kde_one.py 262144 20 > $OUT/lds2b.out 2>&1
echo done
