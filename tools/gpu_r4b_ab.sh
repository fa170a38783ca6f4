#!/usr/bin/env bash
# Round 4, session 2: parts A and B in one call (tools/gpu_r4b_a.sh, tools/gpu_r4b_b.sh).
set -euo pipefail
O=gpurun_out/r4b
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_lifetime.py tests/test_gpu_wal.py --karma-lib bounds > $O/lifetime_wal_bounds.log 2>&1 || [ $? -eq 1 ]  # (a failing test is read afterwards; a crash, abort or time limit ends the script)
tail -1 $O/lifetime_wal_bounds.log
timeout -k 10 600 $T tests -m gpu > $O/r04_gpu_tests.log 2>&1 || [ $? -eq 1 ]  # (a failing test is read afterwards; a crash, abort or time limit ends the script)
tail -1 $O/r04_gpu_tests.log
timeout -k 10 600 $T tests -m gpu --karma-lib bounds > $O/r04_gpu_tests_bounds.log 2>&1 || [ $? -eq 1 ]  # (a failing test is read afterwards; a crash, abort or time limit ends the script)
tail -1 $O/r04_gpu_tests_bounds.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke.log 2>&1
tail -1 $O/r04_smoke.log
timeout -k 10 200 python3 -u tools/replay_study.py --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so --rounds 5 > $O/replay_ab.log 2>&1
cat $O/replay_ab.log
timeout -k 10 300 python3 -u bench.py > $O/r04_bench_default.json 2> $O/r04_bench_default.err
cat $O/r04_bench_default.json
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/r04_bench_driver_style.json 2> $O/r04_bench_driver_style.err
cat $O/r04_bench_driver_style.json
timeout -k 10 300 $T tests/test_gpu_parity.py -k "dynamic_tail or ragged_graph or config3" --karma-lib abbounds > $O/dyn_abbounds.log 2>&1 || [ $? -eq 1 ]  # (a failing test is read afterwards; a crash, abort or time limit ends the script)
tail -1 $O/dyn_abbounds.log
LIBS="units=karma_amd/lib/libkarma_crc32c.so,dyn1=tools/lib/libkarma_crc32c_dyn1.so,dyn2=tools/lib/libkarma_crc32c_dyn2.so,dyn3=tools/lib/libkarma_crc32c_dyn3.so,dyn5=tools/lib/libkarma_crc32c_dyn5.so" \
  timeout -k 10 400 python3 -u tools/ragged_study.py > $O/ragged_dyn_study.log 2>&1
grep -v "first call" $O/ragged_dyn_study.log
LIBS="units=karma_amd/lib/libkarma_crc32c.so,grid2k=tools/lib/libkarma_crc32c_grid.so,grid4k=tools/lib/libkarma_crc32c_t4096.so,grid8k=tools/lib/libkarma_crc32c_t8192.so,gtime_loads=tools/lib/libkarma_crc32c_gtime1.so,gtime_steps=tools/lib/libkarma_crc32c_gtime2.so" \
  timeout -k 10 400 python3 -u tools/ragged_study.py > $O/ragged_grid_study.log 2>&1
grep -v "first call" $O/ragged_grid_study.log
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
for W in ragged segment; do
  timeout -k 10 300 python3 -u bench.py --workload $W > $O/r04_bench_$W.json 2> $O/r04_bench_$W.err
  cat $O/r04_bench_$W.json
done
echo done
