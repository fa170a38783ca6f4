#!/usr/bin/env bash
# Round 4: shipped-configuration builds of the ragged path side by side (byte grid with 2/4/8 KiB
# tiles, the unit plan) on configs[2] and aligned layouts; the one-segment kernel's per-workgroup
# phase stamps (tools build).
set -euo pipefail
O=gpurun_out/r4study
mkdir -p $O
LIBS="t2048=karma_amd/lib/libkarma_crc32c.so,t4096=tools/lib/libkarma_crc32c_t4096.so,t8192=tools/lib/libkarma_crc32c_t8192.so,units=tools/lib/libkarma_crc32c_nogrid.so" \
  timeout -k 10 600 python3 -u tools/ragged_study.py > $O/ragged_study.log 2>&1
grep -v "first call" $O/ragged_study.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 2 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
echo done
