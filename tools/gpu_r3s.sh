# Round 3, session 2: LDS-staged small-record kernel (tools build: KARMA_DIRECT_VARIANT 14 / 15,
# KARMA_WAL_LIST_CRC=1): parity on the bounds-checked tools build first, then timing.
set -e
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "consecutive or bounded_direct" --karma-lib abbounds > gpurun_out/r3s/tests_abbounds.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread -k "listcrc" --karma-lib abbounds > gpurun_out/r3s/tests_wal_abbounds.log 2>&1
timeout -k 10 240 python3 -u tools/direct_study.py --variants 0,14,15 --rounds 4 > gpurun_out/r3s/direct.txt 2>&1
timeout -k 10 240 python3 -u tools/replay_study.py --variants shipped,ab,listcrc --rounds 4 > gpurun_out/r3s/replay.txt 2>&1
echo done
