# round 5: DPP scans in the ragged plan and DPP reductions in the staged kernel -- the bounds build first
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wal.py -m gpu -x -q -k "ragged or config3 or replay or staged or bounded or small" --karma-lib bounds --timeout 200 --timeout-method thread > $O/r05w_bounds.log 2>&1 || exit 10
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05w_gpu_tests.log 2>&1 || exit 11
timeout -k 10 300 python3 -u tools/plan_phases.py --calls 3 --json $O/r05_plan_phases_dpp.json > $O/r05_plan_phases_dpp.log 2>&1 || exit 12
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" ROUNDS=7 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_plan_dpp_ab.txt 2>&1 || exit 13
timeout -k 10 400 python3 -u tools/replay_study.py --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so --rounds 7 --calls 20 > $O/r05_replay_dpp_ab.txt 2>&1 || exit 15
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_dpp -o run -- python3 $OLDPWD/bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $OLDPWD/$O/prof_dpp.log 2>&1 || exit 14
