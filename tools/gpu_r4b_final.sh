#!/usr/bin/env bash
# Round 4 final check: the GPU suite on the shipped, bounds-checked and bounds-checked tools builds,
# smoke(), the default and driver-style bench lines, and the headline kernel's rocprofv3 trace +
# FETCH/WRITE passes.
set -euo pipefail
O=gpurun_out/r4final
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > $O/r04_final_gpu_tests.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/r04_final_gpu_tests.log
timeout -k 10 600 $T tests -m gpu --karma-lib bounds > $O/r04_final_gpu_tests_bounds.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/r04_final_gpu_tests_bounds.log
timeout -k 10 600 $T tests -m gpu --karma-lib abbounds > $O/r04_final_gpu_tests_abbounds.log 2>&1 || [ $? -eq 1 ]
tail -1 $O/r04_final_gpu_tests_abbounds.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_final_smoke.log 2>&1
tail -1 $O/r04_final_smoke.log
timeout -k 10 300 python3 -u bench.py > $O/r04_final_bench_default.json 2> $O/r04_final_bench_default.err
cat $O/r04_final_bench_default.json
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/r04_final_bench_driver_style.json 2> $O/r04_final_bench_driver_style.err
cat $O/r04_final_bench_driver_style.json
timeout -k 10 300 python3 -u bench.py --workload wal_replay > $O/r04_final_bench_wal_replay.json 2> $O/r04_final_bench_wal_replay.err
cat $O/r04_final_bench_wal_replay.json
timeout -k 10 600 bash tools/profile_round.sh r04final fixed > gpurun_out/profile_r04final_fixed.log 2>&1
tail -1 gpurun_out/profile_r04final_fixed.log
echo done
