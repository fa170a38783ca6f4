#!/usr/bin/env bash
# tools/gpu_run.sh TAG STEP... -- the GPU-box runner for every gpurun call (from the repo root):
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh r06a tests bench "study=python3 -u tools/replay_study.py ..."'
# Each STEP runs under its own time limit, writes gpurun_out/TAG/<name>.log (bench lines: .json),
# and the first failing step ends the script (no GPU step after a fault, abort or time limit).
# Named steps:
#   tests | tests_bounds | tests_abbounds  the GPU suite on the shipped / bounds / bounds-tools build
#   wal_tests                              the WAL / multi-host GPU tests alone
#   smoke                                  __graft_entry__.smoke()
#   bench                                  bench.py defaults (the driver's N = 1 line)
#   bench_driver                           bench.py --steps 20 --warmup 5 (the driver's command)
#   bench_<workload>                       bench.py --workload <workload>
#   profile_<workload>                     tools/profile_round.sh TAG <workload> (kernel trace + PMC passes)
#   name=COMMAND                           any command (default limit 400 s; name:SECONDS=COMMAND sets it)
set -uo pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
step() {  # name, seconds, command
  local name=$1 secs=$2 cmd=$3 log="$OUT/$1.log"
  case $name in bench*) log="$OUT/$1.json" ;; esac
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2> "$OUT/$name.err"
  local rc=$?
  tail -c 1500 "$log"
  if [ $rc -ne 0 ]; then
    echo "== $name failed: status $rc"; tail -c 3000 "$OUT/$name.err"; exit $rc
  fi
}
for s in "$@"; do
  case $s in
    tests) step tests 900 "$T tests -m gpu" ;;
    tests_bounds) step tests_bounds 900 "$T tests -m gpu --karma-lib bounds" ;;
    tests_abbounds) step tests_abbounds 900 "$T tests -m gpu --karma-lib abbounds" ;;
    wal_tests) step wal_tests 400 "$T tests/test_gpu_wal.py tests/test_gpu_wal_api.py tests/test_gpu_multi_host.py -m gpu" ;;
    smoke) step smoke 300 "python3 -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
    bench) step bench 600 "python3 -u bench.py" ;;
    bench_driver) step bench_driver 300 "python3 -u bench.py --steps 20 --warmup 5" ;;
    *=*)  # (before the bench_* / profile_* names: a custom step's name may start with them)
      lhs=${s%%=*}; cmd=${s#*=}; name=${lhs%%:*}; secs=400
      [ "$lhs" != "$name" ] && secs=${lhs#*:}
      step "$name" "$secs" "$cmd" ;;
    bench_*) step "$s" 400 "python3 -u bench.py --workload ${s#bench_}" ;;
    profile_*) step "$s" 600 "bash tools/profile_round.sh $TAG ${s#profile_}" ;;
    *) echo "unknown step: $s"; exit 2 ;;
  esac
done
echo "== all steps done"
