#!/usr/bin/env bash
# Round 4: the byte grid against the unit plan on configs[2] and aligned layouts (wave logs and
# interleaved call/kernel times, the tools build), after its tests on the bounds-checked build;
# the lifetime probe.
set -euo pipefail
O=gpurun_out/r4ragged
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_grid.py --karma-lib abbounds > $O/grid_abbounds.log 2>&1
tail -1 $O/grid_abbounds.log
timeout -k 10 400 python3 -u tools/ragged_gap.py --case fixed,config3,config3:nogrid,ragged4k,ragged4k:nogrid --json $O/ragged_gap.json > $O/ragged_gap.log 2>&1
cat $O/ragged_gap.log
timeout -k 10 400 python3 -u tools/ragged_study.py > $O/ragged_study.log 2>&1
cat $O/ragged_study.log
timeout -k 10 200 python3 -u tools/lifetime_probe.py 100 > $O/lifetime_probe.log 2>&1
cat $O/lifetime_probe.log
echo done
