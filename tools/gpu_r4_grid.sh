#!/usr/bin/env bash
# Round 4: the ragged byte grid, the one-segment kernel and the resource-lifetime API on the box --
# their tests on the bounds-checked builds first (a wrong address is reported, not faulted), then
# the shipped build, the configs[2] ragged and configs[3] segment bench lines, the segment A/B, and
# the whole GPU suite.
set -euo pipefail
O=gpurun_out/r4grid
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
NEW="tests/test_gpu_grid.py tests/test_gpu_lifetime.py tests/test_gpu_multi_host.py"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "segment_once or stream_" --karma-lib abbounds > $O/seg_abbounds.log 2>&1
timeout -k 10 120 python3 -u tools/lifetime_probe.py 300 > $O/lifetime_probe.log 2>&1
cat $O/lifetime_probe.log
timeout -k 10 400 $T $NEW --karma-lib abbounds -k "not thousand" > $O/new_tests_abbounds.log 2>&1
timeout -k 10 400 $T $NEW tests/test_gpu_parity.py -k "(segment_once or stream_ or grid or lifetime or multi) and not thousand" > $O/new_tests.log 2>&1
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_ragged.json 2> $O/bench_ragged.err
cat $O/bench_ragged.json
timeout -k 10 300 python3 -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_segment.json 2> $O/bench_segment.err
cat $O/bench_segment.json
timeout -k 10 300 python3 -u tools/segment_once_ab.py --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
timeout -k 10 900 $T tests -m gpu > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
echo done
