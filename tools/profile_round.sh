#!/usr/bin/env bash
# tools/profile_round.sh ROUND -- run on the GPU box (via gpurun) from the repo root.
#
#  1. plain bench line                                  -> gpurun_out/prof/bench_<ROUND>.json
#  2. rocprofv3 --kernel-trace --stats of the same cmd  -> gpurun_out/prof/trace_<ROUND>/...
#  3. rocprofv3 --pmc FETCH_SIZE  (own pass)            -> gpurun_out/prof/pmc_fetch_<ROUND>/...
#  4. rocprofv3 --pmc WRITE_SIZE  (own pass)            -> gpurun_out/prof/pmc_write_<ROUND>/...
# Every GPU step has its own time limit and the steps are chained with &&.
set -euo pipefail
ROUND=${1:-r01}
WL=${2:-fixed}
OUT=gpurun_out/prof
mkdir -p "$OUT"
REPO=$(pwd)
export TMPDIR=/tmp
CMD=(python3 "$REPO/bench.py" --workload "$WL" --steps 300 --warmup 30)
timeout -k 10 300 "${CMD[@]}" > "$OUT/bench_${ROUND}_${WL}.json"
cat "$OUT/bench_${ROUND}_${WL}.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT/trace_${ROUND}_${WL}" -o run \
    -- python3 "$REPO/bench.py" --workload "$WL" --steps 300 --warmup 30 --no-cpu-baseline > "$REPO/$OUT/trace_${ROUND}_${WL}.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$REPO/$OUT/pmc_fetch_${ROUND}_${WL}" -o run \
    -- python3 "$REPO/bench.py" --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline > "$REPO/$OUT/pmc_fetch_${ROUND}_${WL}.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$REPO/$OUT/pmc_write_${ROUND}_${WL}" -o run \
    -- python3 "$REPO/bench.py" --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline > "$REPO/$OUT/pmc_write_${ROUND}_${WL}.log" 2>&1
cd "$REPO"
find "$OUT" -name "*.csv" | head -50
