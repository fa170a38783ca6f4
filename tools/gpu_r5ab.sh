# round 5: the walkers' max and the fused gather plan's sums through DPP
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py tests/test_gpu_wal_api.py tests/test_gpu_multi_host.py -m gpu -x -q --karma-lib bounds --timeout 200 --timeout-method thread > $O/r05ab_wal_bounds.log 2>&1 || exit 10
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05ab_gpu_tests.log 2>&1 || exit 11
timeout -k 10 400 python3 -u tools/replay_study.py --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so --rounds 7 --calls 20 > $O/r05_replay_walkgather_dpp_ab.txt 2>&1 || exit 15
