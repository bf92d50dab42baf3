#!/bin/bash
# Interleaved A/B of library variants (tools/build_variant.sh):
#   bash tools/varrun.sh OUT "N d reps" LIB [LIB ...]   (SCRIPT=tools/lz_time.py
#   for the LocalTransition pass; default tools/kde_time.py)
set -e
OUT=gpurun_out/$1; shift
ARGS=$1; shift
mkdir -p "$OUT"
for r in 1 2; do
  for L in "$@"; do
    # shellcheck disable=SC2086
    timeout -k 10 150 python3 -u tools/lib_ab.py "$L" ${SCRIPT:-tools/kde_time.py} $ARGS >> "$OUT/kde.txt" 2>&1
  done
done
grep "N=" "$OUT/kde.txt"
