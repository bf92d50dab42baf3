#!/bin/bash
# Round-2 first GPU call: full-size KDE parity + VALU/MFMA PMC passes.
set -e -o pipefail
OUT=gpurun_out/r02a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -k "kde or fullsize or guard or pnorm" > $OUT/fullsize.txt 2>&1
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE -T -f csv -d $OUT/pmcA -o run -- python3 $BENCH > $OUT/pmcA.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -f csv -d $OUT/pmcB -o run -- python3 $BENCH > $OUT/pmcB.out 2>&1
echo done
