set -e
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "consecutive or bounded_direct" --karma-lib abbounds > gpurun_out/r3s/tests_fold.log 2>&1
timeout -k 10 240 python3 -u tools/direct_study.py --variants 0,20 --rounds 4 > gpurun_out/r3s/direct_fold.txt 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped --rounds 4 > gpurun_out/r3s/replay_fold.txt 2>&1
echo done
