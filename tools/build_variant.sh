#!/bin/bash
# Build a compile-time variant of the MFMA KDE unit into its own library
# (same-box A/B through tools/lib_ab.py; build_var/ is git-ignored):
#   tools/build_variant.sh NAME "-DABC_KDE_...=... ..."
set -e
cd "$(dirname "$0")/../pyabc_amd/csrc"
make -j8 > /dev/null
OUT=../../build_var
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize $2 -c kde_mfma.hip -o $OUT/kde_mfma_$1.o
objs=$(ls ../_lib/obj/*.o | grep -v kde_mfma.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libabc_$1.so $objs $OUT/kde_mfma_$1.o
echo "$OUT/libabc_$1.so"
