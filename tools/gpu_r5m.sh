# round 5: the ragged units kernel's timing forms (no lookups / no fold) and unit sizes 2-8 KiB
set -o pipefail
O=gpurun_out
mkdir -p $O
LIBS="ship=karma_amd/lib/libkarma_crc32c.so,ab=tools/lib/libkarma_crc32c_ab.so,nolookup=tools/lib/libkarma_crc32c_ab.so@KARMA_RAGGED_UNITS_MODE=1,nofold=tools/lib/libkarma_crc32c_ab.so@KARMA_RAGGED_UNITS_MODE=2,neither=tools/lib/libkarma_crc32c_ab.so@KARMA_RAGGED_UNITS_MODE=3,u4k=tools/lib/libkarma_crc32c_u4096.so,u2k=tools/lib/libkarma_crc32c_u2048.so" ROUNDS=5 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_units_modes.txt 2>&1 || exit 13
