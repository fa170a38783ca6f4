# round 5: the fixed kernel's loop over 2 KiB ragged units from descriptors, against the shipped kernel on 2 and 8 KiB units
set -o pipefail
O=gpurun_out
mkdir -p $O
AB2=tools/lib/libkarma_crc32c_abu2k.so
LAYOUTS="aligned 4096,config3" LIBS="ship=karma_amd/lib/libkarma_crc32c.so,u2k=tools/lib/libkarma_crc32c_u2048.so,u2kfxdesc=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=1,u2kfxarith=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=2" ROUNDS=9 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_units_fixedloop3.txt 2>&1 || exit 13
