#!/usr/bin/env bash
# tools/scan_block_ab.sh -- A/B of the ragged scan/desc block size (KARMA_SCAN_BLOCK) across
# builds (run on the GPU box from the repo root).  Build the alternatives first, here:
#   for B in 256 512; do make -C karma_amd/csrc OBJDIR=$PWD/build/objsb$B \
#       LIBDIR=$PWD/build/libsb$B EXTRA=-DKARMA_SCAN_BLOCK=$B; done
# The shipped library is swapped out for an alternative in the box's scratch copy only.
set -euo pipefail
LIB=karma_amd/lib/libkarma_crc32c.so
cp "$LIB" /tmp/lib_default.so
for B in ${ALTS:-sb256 sb512}; do  # parity first: the ragged GPU tests on each alternative
  cp build/lib$B/libkarma_crc32c.so "$LIB"
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k ragged -x -q --timeout 120 --timeout-method thread > gpurun_out/sb_${B}_parity.log 2>&1
done
for pass in 1 2; do
  cp /tmp/lib_default.so "$LIB"
  ROUNDS=6 RAGGED_VARIANTS="${RV:-}" FIXED_VARIANTS="" timeout -k 10 300 python3 -u tools/ragged_study.py > gpurun_out/sb_1024_$pass.log 2>&1
  for B in ${ALTS:-sb256 sb512}; do
    cp build/lib$B/libkarma_crc32c.so "$LIB"
    ROUNDS=6 RAGGED_VARIANTS="${RV:-}" FIXED_VARIANTS="" timeout -k 10 300 python3 -u tools/ragged_study.py > gpurun_out/sb_${B}_$pass.log 2>&1
  done
done
cp /tmp/lib_default.so "$LIB"
