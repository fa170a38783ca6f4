# round 5: k_units_fixed's loop (stream_unit, LDS-counter wave-steps) over the ragged units, from descriptors or arithmetic
set -o pipefail
O=gpurun_out
mkdir -p $O
AB=tools/lib/libkarma_crc32c_ab.so
AB2=tools/lib/libkarma_crc32c_abu2k.so
LAYOUTS="aligned 4096,aligned 2048" LIBS="ship=karma_amd/lib/libkarma_crc32c.so,fxdesc=$AB@KARMA_RAGGED_UNITS_FIXEDLOOP=1,u2k=$AB2,u2kfxdesc=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=1,u2kfxarith=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=2" ROUNDS=5 timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_units_fixedloop.txt 2>&1 || exit 13
