set -e
mkdir -p gpurun_out/r3s
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread --karma-lib abbounds > gpurun_out/r3s/tests_wal_abbounds2.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s/tests_wal2.log 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,sep,sepdirect4,listcrc --rounds 4 --single > gpurun_out/r3s/replay3.txt 2>&1
echo done
