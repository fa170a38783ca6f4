# round 5: the fixed-loop ragged form with the fixed kernel's LDS allocation / head-tail loads (2 KiB units)
set -o pipefail
O=gpurun_out
mkdir -p $O
AB2=tools/lib/libkarma_crc32c_abu2k.so
LAYOUTS="aligned 4096" LIBS="ship=karma_amd/lib/libkarma_crc32c.so,fxarith=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=2,fxarith_biglds=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=3,fxarith_ht=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=4,fxdesc_biglds=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=5,fxdesc=$AB2@KARMA_RAGGED_UNITS_FIXEDLOOP=1" ROUNDS=7 timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_units_fixedloop2.txt 2>&1 || exit 13
