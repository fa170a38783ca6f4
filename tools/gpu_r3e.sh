set -e
mkdir -p gpurun_out/r3e
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/r3e/stream_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r3e/segment.json 2> gpurun_out/r3e/segment.err
timeout -k 10 200 python -u tools/direct_study.py --variants 0,11,12,13 --rounds 4 > gpurun_out/r3e/direct180.log 2>&1
timeout -k 10 200 python -u tools/direct_study.py --variants 0,11,12,13 --rounds 3 --size 500 --n 400000 > gpurun_out/r3e/direct500.log 2>&1
timeout -k 10 400 python -u tools/ragged_gap.py --case fixed,config3,config3:21@16,config3:21@32,config3:21@64,config3:21@128,config3:26@32,config3,config3:21@32,ragged1k,ragged1k:21@32 --json gpurun_out/r3e/gap5.json > gpurun_out/r3e/gap5.log 2>&1
echo done
