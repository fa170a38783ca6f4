# round 5: flat units kernel on 2 KiB units (the fixed kernel's unit size and step addresses on aligned 4 KiB records)
set -o pipefail
O=gpurun_out
mkdir -p $O
AB=tools/lib/libkarma_crc32c_abu2k.so
LIBS="ship=karma_amd/lib/libkarma_crc32c.so,u2k=tools/lib/libkarma_crc32c_u2048.so,u2kflat8=$AB@KARMA_RAGGED_UNITS_FLAT=8,u2kflat4=$AB@KARMA_RAGGED_UNITS_FLAT=4,u2kneither=$AB@KARMA_RAGGED_UNITS_FLAT=83,u2kflat8nodyn=$AB@KARMA_RAGGED_UNITS_FLAT=8;KARMA_RAGGED_DYN=0,u2knodyn=$AB@KARMA_RAGGED_DYN=0" ROUNDS=5 timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_units_flat_u2k.txt 2>&1 || exit 13
