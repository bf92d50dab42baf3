#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/cdf
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "cdf or resample or propose" > $OUT/tests.txt 2>&1
timeout -k 10 120 python3 tools/probes/cdf_probe.py > $OUT/probe.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tr -o run -- python3 tools/probes/cdf_probe.py > $OUT/probe_prof.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $OUT/tr2 -o run -- python3 tools/probes/cdf_scale.py > $OUT/scale.txt 2>&1
echo done
