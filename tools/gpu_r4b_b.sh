#!/usr/bin/env bash
# Round 4, session 2, part B: the ragged byte grid (2/4/8 KiB tile builds) against the shipped unit
# plan, side by side in one process; the one-segment kernel against the looping fused kernel; the
# other workloads' bench lines.
set -euo pipefail
O=gpurun_out/r4b
mkdir -p $O
LIBS="units=karma_amd/lib/libkarma_crc32c.so,grid2k=tools/lib/libkarma_crc32c_grid.so,grid4k=tools/lib/libkarma_crc32c_t4096.so,grid8k=tools/lib/libkarma_crc32c_t8192.so,gtime_loads=tools/lib/libkarma_crc32c_gtime1.so,gtime_steps=tools/lib/libkarma_crc32c_gtime2.so" \
  timeout -k 10 500 python3 -u tools/ragged_study.py > $O/ragged_grid_study.log 2>&1
grep -v "first call" $O/ragged_grid_study.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
for W in ragged segment stream wal_replay host; do
  timeout -k 10 300 python3 -u bench.py --workload $W > $O/r04_bench_$W.json 2> $O/r04_bench_$W.err
  cat $O/r04_bench_$W.json
done
echo done
