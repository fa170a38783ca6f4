set -e
mkdir -p gpurun_out/r3s
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread --karma-lib abbounds > gpurun_out/r3s/tests_wal_direct2.log 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,nodirect --rounds 4 --single > gpurun_out/r3s/replay6.txt 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --mix config3 --variants shipped,nodirect --rounds 3 > gpurun_out/r3s/replay6_mix.txt 2>&1
echo done
