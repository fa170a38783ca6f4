#!/usr/bin/env bash
# Round 4, session 2, part B: the dynamic-tail ragged test on the bounds-checked tools build; the
# ragged unit plan with a dynamic tail (dyn builds) and the byte grid (2/4/8 KiB tile builds, its
# timing builds) against the shipped unit plan, side by side in one process; the one-segment
# kernel against the looping fused kernel; the ragged and segment bench lines.
set -euo pipefail
O=gpurun_out/r4b
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "dynamic_tail or ragged_graph or config3" --karma-lib abbounds > $O/dyn_abbounds.log 2>&1
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
