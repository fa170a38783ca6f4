set -e
mkdir -p gpurun_out/r3s
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread --karma-lib abbounds > gpurun_out/r3s/tests_wal_direct3.log 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,nodirect --rounds 3 --size 1000 --count 200000 > gpurun_out/r3s/replay_1k.txt 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,nodirect --rounds 3 --size 3000 --count 60000 > gpurun_out/r3s/replay_3k.txt 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped --rounds 3 > gpurun_out/r3s/replay_180_after.txt 2>&1
echo done
