#!/usr/bin/env bash
# Round 4: the one-segment kernel with its table loads ordered ahead of every chunk load (stamps,
# bench line, rocprofv3 trace), its tests on the bounds build; the byte grid's timing builds
# (loads alone / unmasked steps) beside the shipped grid and the unit plan.
set -euo pipefail
O=gpurun_out/r4seg2
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "segment_once or stream_" --karma-lib bounds > $O/seg_bounds.log 2>&1
tail -1 $O/seg_bounds.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 2 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o seg -- python3 -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_segment_prof.json 2> $O/bench_segment_prof.err
cat $O/bench_segment_prof.json
find $O/prof -name "*kernel_stats.csv" -exec head -3 {} \;
LIBS="t2048=karma_amd/lib/libkarma_crc32c.so,gtime1=tools/lib/libkarma_crc32c_gtime1.so,gtime2=tools/lib/libkarma_crc32c_gtime2.so,units=tools/lib/libkarma_crc32c_nogrid.so" \
  timeout -k 10 600 python3 -u tools/ragged_study.py > $O/ragged_timing.log 2>&1
grep -v "first call" $O/ragged_timing.log

timeout -k 10 300 python3 -u bench.py --workload wal_replay --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_wal_replay.json 2> $O/bench_wal_replay.err
cat $O/bench_wal_replay.json
echo done
