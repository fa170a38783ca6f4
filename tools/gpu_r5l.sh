# round 5: ragged records stepped over whole 16-byte blocks with masked edges (no record reads in plan / finalize)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or config3" --karma-lib bounds --timeout 200 --timeout-method thread > $O/r05l_ragged_bounds.log 2>&1 || exit 10
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05l_gpu_tests.log 2>&1 || exit 11
timeout -k 10 300 python3 -u tools/plan_phases.py --calls 3 --json $O/r05_plan_phases_masked.json > $O/r05_plan_phases_masked.log 2>&1 || exit 12
LIBS="head=tools/lib/libkarma_crc32c_head.so,new=karma_amd/lib/libkarma_crc32c.so" ROUNDS=7 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_masked_edges_ab.txt 2>&1 || exit 13
