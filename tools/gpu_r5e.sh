# round 5: three-input XOR (v_bitop3_b32) in the table steps -- suite, staged probe, replay and ragged A/B
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r05e_gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u tools/staged_probe.py --json $O/r05_staged_probe_xor3.json > $O/r05_staged_probe_xor3.log 2>&1 || exit 11
timeout -k 10 400 python3 -u tools/replay_study.py --variants shipped,lib=tools/lib/libkarma_crc32c_prev.so --rounds 5 > $O/r05_replay_xor3.txt 2>&1 || exit 12
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_ragged_xor3.txt 2>&1 || exit 13
