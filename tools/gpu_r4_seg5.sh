#!/usr/bin/env bash
# Round 4: the one-segment kernel with its tables in LDS before any chunk load (tests on the
# bounds build, stamps, rocprofv3 kernel stats, the segment bench line).
set -euo pipefail
O=gpurun_out/r4seg5
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_lifetime.py -k "segment_once or stream_ or concurrently" --karma-lib bounds > $O/seg_bounds.log 2>&1
tail -1 $O/seg_bounds.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 2 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o seg -- python3 -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_segment_prof.json 2> $O/bench_segment_prof.err
cat $O/bench_segment_prof.json
find $O/prof -name "*kernel_stats.csv" -exec head -3 {} \;
echo done
