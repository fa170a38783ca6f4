#!/usr/bin/env bash
# Round 4, session 2, part D: the chunked dynamic tail (tests on the bounds-checked tools build,
# then the dyn builds against the shipped unit plan); the replay's two round-4 changes taken apart
# (gather blocks per segment, one small-record launch); the lifetime test on the bounds build;
# then part C's profiles (rocprofv3 kernel traces, FETCH/WRITE passes, the replay's SQ passes).
set -euo pipefail
O=gpurun_out/r4d
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "dynamic_tail" --karma-lib abbounds > $O/dyn_abbounds.log 2>&1
tail -1 $O/dyn_abbounds.log
timeout -k 10 200 $T tests/test_gpu_lifetime.py --karma-lib bounds > $O/lifetime_bounds.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/lifetime_bounds.log
LIBS="units=karma_amd/lib/libkarma_crc32c.so,dyn2=tools/lib/libkarma_crc32c_dyn2.so,dyn3=tools/lib/libkarma_crc32c_dyn3.so,dyn5=tools/lib/libkarma_crc32c_dyn5.so" \
  timeout -k 10 400 python3 -u tools/ragged_study.py > $O/ragged_dyn_study.log 2>&1
grep -v "first call" $O/ragged_dyn_study.log
timeout -k 10 300 python3 -u tools/replay_study.py --rounds 5 \
  --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so,ab,ab:KARMA_GATHER_PARTS=1,ab:KARMA_SMALL_WHICH=0 > $O/replay_ab.log 2>&1
cat $O/replay_ab.log
for W in fixed ragged segment; do
  timeout -k 10 600 bash tools/profile_round.sh r04 $W > gpurun_out/profile_r04_$W.log 2>&1
  tail -2 gpurun_out/profile_r04_$W.log
done
timeout -k 10 600 bash tools/pmc_replay.sh r04 > gpurun_out/pmc_replay_r04.log 2>&1
tail -2 gpurun_out/pmc_replay_r04.log
echo done
