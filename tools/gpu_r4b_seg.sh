#!/usr/bin/env bash
# Round 4, session 2: the one-segment kernel with its stride image computed in place and the fold
# tables stored while the chunks are in flight -- its tests on the bounds-checked builds, then a
# same-box A/B against the previous build (session 1's kernel) and the phase stamps.
set -euo pipefail
O=gpurun_out/r4seg
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_lifetime.py -k "segment_once or stream_ or concurrently" --karma-lib abbounds > $O/seg_abbounds.log 2>&1
tail -1 $O/seg_abbounds.log
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_lifetime.py -k "segment_once or stream_ or concurrently" > $O/seg_shipped.log 2>&1
tail -1 $O/seg_shipped.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 8 --libs new=karma_amd/lib/libkarma_crc32c.so,prev=tools/lib/libkarma_crc32c_prev.so --json $O/segment_libs_ab.json > $O/segment_libs_ab.log 2>&1
cat $O/segment_libs_ab.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
timeout -k 10 200 python3 -u bench.py --workload segment --no-cpu-baseline > $O/bench_segment.json 2> $O/bench_segment.err
cat $O/bench_segment.json
echo done
