set -e
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 200 --timeout-method thread -k "several_passes or append_matches" > gpurun_out/r3s/tests_append_passes.log 2>&1
timeout -k 10 400 bash tools/pmc_replay.sh r03s > gpurun_out/r3s/pmc_replay.log 2>&1
echo done
