set -e
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "consecutive or bounded_direct" --karma-lib abbounds > gpurun_out/r3s/tests_skew4.log 2>&1
for sz in 16 56 120 180; do
  timeout -k 10 200 python3 -u tools/direct_study.py --variants 0,20,27 --rounds 3 --size $sz > gpurun_out/r3s/skew4_size$sz.txt 2>&1
done
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped --rounds 4 > gpurun_out/r3s/replay_skew4.txt 2>&1
echo done
