#!/bin/bash
# End-to-end configs (drop-in API) + per-kernel stats of C2 / C4 / C5.
set -e -o pipefail
OUT=gpurun_out/cfg_r02
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
for c in c2 c4 c5; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/stats_$c -o run -- python3 tools/bench_configs.py --only $c > $OUT/$c.jsonl 2> $OUT/$c.err
done
echo done
