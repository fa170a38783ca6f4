# round 5: flat units kernel with arithmetic unit addresses (no descriptors) and without unit-state stores,
# aligned layouts only (the arithmetic form reads arena bytes [u 2 KiB, (u + 1) 2 KiB) for unit u)
set -o pipefail
O=gpurun_out
mkdir -p $O
AB=tools/lib/libkarma_crc32c_abu2k.so
LAYOUTS="aligned 4096,aligned 2048" LIBS="ship=karma_amd/lib/libkarma_crc32c.so,u2k=tools/lib/libkarma_crc32c_u2048.so,flat8=$AB@KARMA_RAGGED_UNITS_FLAT=8,arith=$AB@KARMA_RAGGED_UNITS_FLAT=864,nostore=$AB@KARMA_RAGGED_UNITS_FLAT=8128,neither=$AB@KARMA_RAGGED_UNITS_FLAT=8192" ROUNDS=5 timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_units_flat_arith.txt 2>&1 || exit 13
