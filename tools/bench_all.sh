#!/usr/bin/env bash
# tools/bench_all.sh TAG -- every bench.py workload once (run via gpurun from the repo root);
# one JSON line per workload in gpurun_out/bench_<TAG>_<workload>.json.  Each step has its
# own time limit and a failing step ends the script.
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > "$OUT/bench_${TAG}_${name}.json" 2> "$OUT/bench_${TAG}_${name}.err"
  echo "== $name"; cat "$OUT/bench_${TAG}_${name}.json"
}
run fixed
run ragged --workload ragged
run stream --workload stream
run segment --workload segment
run host --workload host
run wal_append --workload wal_append
run wal_replay --workload wal_replay
run wal_append_mix --workload wal_append --wal-mix config3 --steps 10 --warmup 2
run wal_replay_mix --workload wal_replay --wal-mix config3 --steps 10 --warmup 2
run kfp_encode --workload kfp_encode
run kfp_parse --workload kfp_parse
run config5_slice --records-per-gpu 33554432 --steps 5 --warmup 1 --no-cpu-baseline
