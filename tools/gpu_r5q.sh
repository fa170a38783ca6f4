# round 5: the ragged units kernel timed after another units kernel instead of after the plan (no dynamic tail)
set -o pipefail
O=gpurun_out
mkdir -p $O
AB=tools/lib/libkarma_crc32c_ab.so
LAYOUTS="aligned 4096,config3" LIBS="ab=$AB,nodyn=$AB@KARMA_RAGGED_DYN=0,twice_nodyn=$AB@KARMA_RAGGED_DYN=0;KARMA_RAGGED_UNITS_TWICE=1" ROUNDS=5 timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_units_twice_nodyn.txt 2>&1 || exit 13
