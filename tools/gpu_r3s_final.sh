# Round-3 session-2 final validation of the committed tree: GPU suite (shipped + bounds builds), smoke,
# the default bench line and a driver-style bench line.  Each GPU step has its own limit.
set -e
O=gpurun_out/r3sfinal5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --karma-lib abbounds > $O/gpu_tests_bounds.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_style.json 2> $O/bench_driver_style.err
timeout -k 10 300 python3 -u bench.py --workload wal_replay --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_wal_replay.json 2> $O/bench_wal_replay.err
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped --rounds 4 --single > $O/replay_study.txt 2>&1
echo done
