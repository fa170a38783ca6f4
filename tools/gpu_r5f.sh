# round 5: the two-lanes-per-record staged kernel -- parity (bounds-checked tools build first), probe, replay A/B
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wal.py -m gpu -x -q -k "bounded or pair" --karma-lib abbounds --timeout 120 --timeout-method thread > $O/r05f_pair_abbounds.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wal.py -m gpu -x -q -k "bounded or pair" --timeout 120 --timeout-method thread > $O/r05f_pair_tests.log 2>&1 || exit 11
timeout -k 10 300 python3 -u tools/staged_probe.py --json $O/r05_staged_probe_pair.json > $O/r05_staged_probe_pair.log 2>&1 || exit 12
timeout -k 10 400 python3 -u tools/replay_study.py --variants shipped,ab,ab:KARMA_STAGE_PAIR=1 --rounds 5 > $O/r05_replay_pair.txt 2>&1 || exit 13
