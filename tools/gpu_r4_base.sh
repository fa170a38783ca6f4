#!/usr/bin/env bash
# Round-4 baseline on the box: the configs[2] ragged line and the segment line of the starting tree.
set -euo pipefail
O=gpurun_out/r4base
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_ragged.json 2> $O/bench_ragged.err
timeout -k 10 300 python3 -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_segment.json 2> $O/bench_segment.err
cat $O/bench_ragged.json $O/bench_segment.json
echo done
