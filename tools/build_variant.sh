#!/bin/bash
# Build a compile-time variant of one translation unit into its own library
# (same-box A/B through tools/lib_ab.py; build_var/ is git-ignored):
#   tools/build_variant.sh NAME "FLAGS" [UNIT]   (UNIT: kde_mfma | local_mfma | local)
set -e
cd "$(dirname "$0")/../pyabc_amd/csrc"
make -j8 > /dev/null
OUT=../../build_var
UNIT=${3:-kde_mfma}
mkdir -p $OUT
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function"
if [ "$UNIT" != local ] && [ -z "$AGPR_FORM" ]; then BASE="$BASE -mllvm -amdgpu-mfma-vgpr-form=1"; fi
if [ "$UNIT" = kde_mfma ]; then
  BASE="$BASE -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp"
fi
# shellcheck disable=SC2086
/opt/rocm/bin/hipcc $BASE $2 -c $UNIT.hip -o $OUT/${UNIT}_$1.o
objs=$(ls ../_lib/obj/*.o | grep -v "/$UNIT.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libabc_$1.so $objs $OUT/${UNIT}_$1.o
echo "$OUT/libabc_$1.so"
