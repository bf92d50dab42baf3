#!/bin/bash
# Rebuild the in-tree library, then run one command on the GPU box.
#   tools/gpurun.sh TIMEOUT 'command'
set -e
make -C "$(dirname "$0")/../pyabc_amd/csrc" -j8 > /dev/null
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
