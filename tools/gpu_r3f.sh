set -e
mkdir -p gpurun_out/r3f
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/r3f/stream_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r3f/segment.json 2> gpurun_out/r3f/segment.err
echo done
