#!/usr/bin/env bash
# Round 4, session 2, part E2: the final tree's bench lines (default, the driver's short form, every
# workload the bench has) and its profiles (rocprofv3 kernel traces + FETCH/WRITE passes of the
# fixed, ragged and segment lines; the rotated replay's trace, SQ and FETCH/WRITE passes).
set -euo pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/r04_bench_default.json 2> $O/r04_bench_default.err
cat $O/r04_bench_default.json
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/r04_bench_driver_style.json 2> $O/r04_bench_driver_style.err
cat $O/r04_bench_driver_style.json
for W in ragged segment stream wal_replay wal_append host kfp_parse; do
  timeout -k 10 300 python3 -u bench.py --workload $W > $O/r04_bench_$W.json 2> $O/r04_bench_$W.err
  cat $O/r04_bench_$W.json
done
for W in ragged segment; do
  timeout -k 10 600 bash tools/profile_round.sh r04f $W > gpurun_out/profile_r04f_$W.log 2>&1
  tail -1 gpurun_out/profile_r04f_$W.log
done
timeout -k 10 600 bash tools/pmc_replay.sh r04f > gpurun_out/pmc_replay_r04f.log 2>&1
tail -1 gpurun_out/pmc_replay_r04f.log
echo done
