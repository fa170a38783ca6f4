# round 5: the ragged plan's 64-bit scans and look-back sums through DPP -- the bounds build first
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or config3 or lookback" --karma-lib bounds --timeout 200 --timeout-method thread > $O/r05ad_bounds.log 2>&1 || exit 10
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05ad_gpu_tests.log 2>&1 || exit 11
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" ROUNDS=7 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_plan_lb_dpp_ab.txt 2>&1 || exit 13
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_lbdpp -o run -- python3 $OLDPWD/bench.py --workload ragged --steps 100 --warmup 10 --no-cpu-baseline > $OLDPWD/$O/prof_lbdpp.log 2>&1 || exit 14
