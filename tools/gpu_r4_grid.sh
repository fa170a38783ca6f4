#!/usr/bin/env bash
# Round 4: first GPU runs of the ragged byte grid -- its tests on the bounds-checked builds first
# (a wrong address is reported, not faulted), then on the shipped build, then the ragged bench.
set -euo pipefail
O=gpurun_out/r4grid
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 120 --timeout-method thread --karma-lib abbounds > $O/grid_tests_abbounds.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 120 --timeout-method thread > $O/grid_tests.log 2>&1
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_ragged.json 2> $O/bench_ragged.err
cat $O/bench_ragged.json
echo done
