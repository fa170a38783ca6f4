#!/usr/bin/env bash
# Round 4, session 2, part E1: the shipped dynamic tail (k = 3) and the one-block gather on the
# bounds builds and the shipped build (whole GPU suites), smoke(); then same-box A/Bs against the
# previous builds: ragged (dyn0 = no dynamic tail), replay (the session's first commit), one segment.
set -euo pipefail
O=gpurun_out/r4e
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "dynamic_tail or segment_once or stream_ or ragged" --karma-lib abbounds > $O/abbounds_focus.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/abbounds_focus.log
timeout -k 10 600 $T tests -m gpu > $O/r04_gpu_tests.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/r04_gpu_tests.log
timeout -k 10 600 $T tests -m gpu --karma-lib bounds > $O/r04_gpu_tests_bounds.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/r04_gpu_tests_bounds.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke.log 2>&1
tail -1 $O/r04_smoke.log
LIBS="dyn3=karma_amd/lib/libkarma_crc32c.so,dyn0=tools/lib/libkarma_crc32c_dyn0.so" \
  timeout -k 10 300 python3 -u tools/ragged_study.py > $O/ragged_dyn_study.log 2>&1
grep -v "first call" $O/ragged_dyn_study.log
timeout -k 10 200 python3 -u tools/replay_study.py --rounds 5 --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so > $O/replay_ab.log 2>&1
cat $O/replay_ab.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --libs new=karma_amd/lib/libkarma_crc32c.so,prev=tools/lib/libkarma_crc32c_prev.so --json $O/segment_libs_ab.json > $O/segment_libs_ab.log 2>&1
cat $O/segment_libs_ab.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,1 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
echo done
