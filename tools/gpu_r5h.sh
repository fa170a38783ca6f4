# round 5: per-round partial runs in the plan -- ragged tests (bounds build first), A/B against R = 1 and the round's start
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or config3" --karma-lib bounds --timeout 120 --timeout-method thread > $O/r05h_ragged_bounds.log 2>&1 || exit 10
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r05h_gpu_tests.log 2>&1 || exit 11
LIBS="new=karma_amd/lib/libkarma_crc32c.so,r1=tools/lib/libkarma_crc32c_r1.so,prev=tools/lib/libkarma_crc32c_prev.so" timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05h_ragged.txt 2>&1 || exit 12
