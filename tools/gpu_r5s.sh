# round 5: finalize's unit-state loads issued before its table stores (one round trip fewer)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or config3" --timeout 200 --timeout-method thread > $O/r05s_ragged_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u tools/plan_phases.py --calls 3 --json $O/r05_plan_phases_fin2.json > $O/r05_plan_phases_fin2.log 2>&1 || exit 12
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" ROUNDS=7 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_finalize_overlap_ab.txt 2>&1 || exit 13
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_fin2 -o run -- python3 $OLDPWD/bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $OLDPWD/$O/prof_fin2.log 2>&1 || exit 14
