#!/bin/bash
# Round 3 (re-entry): whole -m gpu suite + smoke on HEAD, the round profile
# (kernel stats + PMC passes of the headline bench), the bench line, configs.
set -e -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/gpu_all.txt 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
bash tools/gpu_profile.sh r03 > $OUT/profile.txt 2>&1
timeout -k 10 400 python3 -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
echo done
