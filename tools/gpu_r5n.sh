# round 5: the ragged units kernel as one chunk stream per wave (k_units_ragged_flat, tools build)
set -o pipefail
O=gpurun_out
mkdir -p $O
AB=tools/lib/libkarma_crc32c_ab.so
LIBS="ship=karma_amd/lib/libkarma_crc32c.so,flat8=$AB@KARMA_RAGGED_UNITS_FLAT=8,flat4=$AB@KARMA_RAGGED_UNITS_FLAT=4,flat8neither=$AB@KARMA_RAGGED_UNITS_FLAT=83" ROUNDS=5 timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_units_flat.txt 2>&1 || exit 13
