#!/bin/bash
# Round profile on one MI355X: kernel stats + PMC passes (one counter group
# per pass, as MI355X_MICROARCH.md's rocprofv3 section prescribes) over the
# headline bench, plus the per-kernel roofline table.
#   /usr/local/graft/bin/gpurun -- 'bash tools/gpu_profile.sh r02'
set -e -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/stats -o run -- python3 $BENCH > $OUT/bench_stats.json 2> $OUT/bench_stats.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/write -o run -- python3 $BENCH > $OUT/bench_write.json 2> $OUT/bench_write.err
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE -T -f csv -d $OUT/pmcA -o run -- python3 $BENCH > $OUT/pmcA.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -f csv -d $OUT/pmcB -o run -- python3 $BENCH > $OUT/pmcB.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -T -f csv -d $OUT/pmcC -o run -- python3 $BENCH > $OUT/pmcC.out 2>&1
timeout -k 10 300 python3 -u tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err
echo "profile $TAG done"
