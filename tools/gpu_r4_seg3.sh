#!/usr/bin/env bash
# Round 4: the one-segment kernel reading the call tag late (wave 0 only): tests (bounds build),
# phase stamps, rocprofv3 kernel stats of the segment bench.
set -euo pipefail
O=gpurun_out/r4seg3
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_lifetime.py -k "segment_once or stream_ or concurrently" --karma-lib bounds > $O/seg_bounds.log 2>&1
tail -1 $O/seg_bounds.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 2 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o seg -- python3 -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_segment_prof.json 2> $O/bench_segment_prof.err
cat $O/bench_segment_prof.json
find $O/prof -name "*kernel_stats.csv" -exec head -3 {} \;
timeout -k 10 300 $T tests/test_gpu_grid.py --karma-lib abbounds > $O/grid_abbounds.log 2>&1
tail -1 $O/grid_abbounds.log
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_ragged.json 2> $O/bench_ragged.err
cat $O/bench_ragged.json
timeout -k 10 300 python3 -u bench.py --workload wal_replay --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_wal_replay.json 2> $O/bench_wal_replay.err
cat $O/bench_wal_replay.json
echo done
