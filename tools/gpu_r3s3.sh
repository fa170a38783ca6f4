set -e
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "consecutive or bounded_direct" --karma-lib abbounds > gpurun_out/r3s/tests_abbounds4.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread --karma-lib abbounds > gpurun_out/r3s/tests_wal_abbounds3.log 2>&1
timeout -k 10 240 python3 -u tools/direct_study.py --variants 0,20,22 --rounds 3 > gpurun_out/r3s/direct7.txt 2>&1
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,inline,sepdirect4 --rounds 4 --single > gpurun_out/r3s/replay4.txt 2>&1
timeout -k 10 300 python3 -u bench.py --workload wal_replay --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3s/bench_wal_replay.json 2> gpurun_out/r3s/bench_wal_replay.err
timeout -k 10 400 bash tools/pmc_small.sh r03s && echo done
