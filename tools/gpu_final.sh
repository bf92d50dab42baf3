#!/bin/bash
# Round-2 final check: whole -m gpu suite, smoke, rocprofv3 kernel stats +
# PMC passes of the headline bench, the bench line with its CPU baseline,
# and the end-to-end configs.
set -e -o pipefail
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/gpu_all.txt 2>&1
cp gpurun_out/kde_fullsize_parity.json $OUT/
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
bash tools/gpu_profile.sh r02 > $OUT/profile.txt 2>&1
python3 tools/pmc_traffic.py gpurun_out/prof_r02 r02 > $OUT/pmc_traffic.txt 2>&1
python3 tools/kde_pmc.py gpurun_out/prof_r02 r02 > $OUT/kde_pmc.txt 2>&1
cp profiles/kde_traffic.json profiles/r02_kde_pmc.json profiles/r02_pmc_summary.csv $OUT/
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 python3 -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
echo done
