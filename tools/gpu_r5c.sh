set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r05c_gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u tools/plan_phases.py --calls 5 --json $O/r05_plan_phases_new.json > $O/r05_plan_phases_new.log 2>&1 || exit 11
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_plan_study.txt 2>&1 || exit 12
