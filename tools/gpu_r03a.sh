#!/bin/bash
# Round 3, first call: the whole -m gpu suite on HEAD (incl. the new C5
# full-size KDE parity test), smoke, and PMC passes over the d > 8 default
# (kde_mfma_lds2f_kernel) at N = M = 262144, d = 20.
set -e -o pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/gpu_all.txt 2>&1
cp gpurun_out/kde_fullsize_parity.json $OUT/
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d $OUT/pmc20a -o run -- python3 tools/kde_one.py 262144 20 > $OUT/pmc20a.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C2 -T -f csv -d $OUT/pmc20b -o run -- python3 tools/kde_one.py 262144 20 > $OUT/pmc20b.out 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/stats20 -o run -- python3 tools/kde_one.py 262144 20 > $OUT/stats20.out 2>&1
echo done
