#!/usr/bin/env bash
# tools/ragged_unit_ab.sh -- A/B of the ragged unit size across two builds (run on the GPU box).
# Build the alternative first, here:  make -C karma_amd/csrc OBJDIR=$PWD/build/obj4k \
#     LIBDIR=$PWD/build/lib4k EXTRA=-DKARMA_RAGGED_UNIT=4096
# The shipped library is swapped out for the alternative in the box's scratch copy only.
set -euo pipefail
LIB=karma_amd/lib/libkarma_crc32c.so
cp "$LIB" /tmp/lib_default.so
for pass in 1 2; do
  cp /tmp/lib_default.so "$LIB"
  ROUNDS=6 RAGGED_VARIANTS="${RV:-1 3}" FIXED_VARIANTS="" timeout -k 10 300 python3 -u tools/ragged_study.py > gpurun_out/rua_8k_$pass.log 2>&1
  cp build/lib4k/libkarma_crc32c.so "$LIB"
  ROUNDS=6 RAGGED_VARIANTS="${RV:-1 3}" FIXED_VARIANTS="" timeout -k 10 300 python3 -u tools/ragged_study.py > gpurun_out/rua_4k_$pass.log 2>&1
done
cp /tmp/lib_default.so "$LIB"
