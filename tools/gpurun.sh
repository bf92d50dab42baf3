#!/bin/bash
# Rebuild the in-tree library here, then run tools/gpu_job.sh on the GPU box.
#   tools/gpurun.sh TIMEOUT NAME STEP [STEP ...]     (steps: tools/gpu_job.sh)
set -e
make -C "$(dirname "$0")/../pyabc_amd/csrc" -j8 > /dev/null
T=$1
shift
cmd="bash tools/gpu_job.sh"
for a in "$@"; do cmd+=" $(printf %q "$a")"; done
exec /usr/local/graft/bin/gpurun --timeout "$T" -- "$cmd"
