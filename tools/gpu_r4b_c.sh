#!/usr/bin/env bash
# Round 4, session 2, part C: rocprofv3 kernel traces and FETCH/WRITE passes (each its own run) for
# the fixed (headline), ragged and segment bench lines; the rotated replay's trace, SQ and FETCH/WRITE passes.
set -euo pipefail
for W in fixed ragged segment; do
  timeout -k 10 600 bash tools/profile_round.sh r04 $W > gpurun_out/profile_r04_$W.log 2>&1
  tail -3 gpurun_out/profile_r04_$W.log
done
timeout -k 10 600 bash tools/pmc_replay.sh r04 > gpurun_out/pmc_replay_r04.log 2>&1
tail -2 gpurun_out/pmc_replay_r04.log
echo done
