#!/usr/bin/env bash
# tools/profile_all.sh ROUND -- the round's committed profiles (run via gpurun from the repo root):
# bench line + rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes for the fixed, ragged and
# stream workloads (tools/profile_round.sh), kernel stats for the segment-latency and WAL replay
# workloads.  Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
ROUND=${1:-r01}
REPO=$(pwd)
for WL in fixed ragged stream; do
  bash tools/profile_round.sh "$ROUND" "$WL"
done
OUT=gpurun_out/prof
export TMPDIR=/tmp
for WL in segment wal_replay; do
  timeout -k 10 300 python3 bench.py --workload "$WL" --steps 20 --warmup 3 > "$OUT/bench_${ROUND}_${WL}.json"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT/trace_${ROUND}_${WL}" -o run \
      -- python3 "$REPO/bench.py" --workload "$WL" --steps 20 --warmup 3 --no-cpu-baseline \
      > "$REPO/$OUT/trace_${ROUND}_${WL}.log" 2>&1
  cd "$REPO"
done
echo done
