#!/usr/bin/env bash
# Round 4, session 2, part A: the lifetime and WAL tests on the bounds build, then the GPU suite on
# the shipped and bounds builds, smoke(), the default and driver-style bench lines, and the
# device-resident replay against the previous commit's library.
set -euo pipefail
O=gpurun_out/r4b
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_lifetime.py tests/test_gpu_wal.py --karma-lib bounds > $O/lifetime_wal_bounds.log 2>&1
tail -1 $O/lifetime_wal_bounds.log
timeout -k 10 600 $T tests -m gpu > $O/r04_gpu_tests.log 2>&1
tail -1 $O/r04_gpu_tests.log
timeout -k 10 600 $T tests -m gpu --karma-lib bounds > $O/r04_gpu_tests_bounds.log 2>&1
tail -1 $O/r04_gpu_tests_bounds.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke.log 2>&1
tail -1 $O/r04_smoke.log
timeout -k 10 200 python3 -u tools/replay_study.py --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so --rounds 5 > $O/replay_ab.log 2>&1
cat $O/replay_ab.log
timeout -k 10 300 python3 -u bench.py > $O/r04_bench_default.json 2> $O/r04_bench_default.err
cat $O/r04_bench_default.json
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/r04_bench_driver_style.json 2> $O/r04_bench_driver_style.err
cat $O/r04_bench_driver_style.json
echo done
