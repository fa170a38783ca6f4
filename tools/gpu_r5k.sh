# round 5: the plan reordered (offsets with the ticket, look-back before the edge loads)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or config3" --timeout 200 --timeout-method thread > $O/r05k_ragged_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u tools/plan_phases.py --calls 3 --json $O/r05_plan_phases_reorder.json > $O/r05_plan_phases_reorder.log 2>&1 || exit 11
LIBS="head=tools/lib/libkarma_crc32c_head.so,new=karma_amd/lib/libkarma_crc32c.so" ROUNDS=7 timeout -k 10 500 python3 -u tools/ragged_study.py > $O/r05_plan_reorder_ab.txt 2>&1 || exit 12
