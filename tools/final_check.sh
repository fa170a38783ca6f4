#!/usr/bin/env bash
# tools/final_check.sh TAG -- the round-end checks on the GPU box (via gpurun, from the repo root):
# the GPU suite on the shipped, the bounds-checked and the bounds-checked tools build, smoke(), the default bench line and a
# driver-style short run.  Each step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --karma-lib bounds > "$OUT/gpu_tests_bounds.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --karma-lib abbounds > "$OUT/gpu_tests_abbounds.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver_style.json" 2> "$OUT/bench_driver_style.err"
echo done
