# round-3 checks of the fused replay / fused stream combine / size-0 (run from the repo root on the GPU box)
set -e
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest tests/test_gpu_wal.py tests/test_gpu_wal_api.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d/wal_tests.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/r3d/stream_tests.log 2>&1
timeout -k 10 300 python -u tools/replay_study.py --variants shipped,sep --single --rounds 3 > gpurun_out/r3d/replay.log 2>&1
timeout -k 10 300 python -u bench.py --workload segment --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r3d/segment.json 2> gpurun_out/r3d/segment.err
echo done
