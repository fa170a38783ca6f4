#!/usr/bin/env bash
# Round 4: the ragged byte grid and the resource-lifetime API on the box -- their tests on the
# bounds-checked builds first (a wrong address is reported, not faulted), then the shipped build,
# the whole GPU suite, and the configs[2] ragged bench line.
set -euo pipefail
O=gpurun_out/r4grid
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_grid.py tests/test_gpu_lifetime.py tests/test_gpu_multi_host.py --karma-lib abbounds > $O/new_tests_abbounds.log 2>&1
timeout -k 10 300 $T tests/test_gpu_grid.py tests/test_gpu_lifetime.py tests/test_gpu_multi_host.py > $O/new_tests.log 2>&1
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_ragged.json 2> $O/bench_ragged.err
cat $O/bench_ragged.json
timeout -k 10 900 $T tests -m gpu > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
echo done
