# round 5: walk candidates written per round (build knob KARMA_WALK_DIRECT_PUT=1) -- bounds build first
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u tools/replay_study.py --variants lib=tools/lib/libkarma_crc32c_wdpbounds.so --rounds 1 --calls 3 > $O/r05ac_wdp_bounds.txt 2>&1 || exit 10
timeout -k 10 300 python3 -u tools/replay_study.py --mix config3 --variants lib=tools/lib/libkarma_crc32c_wdpbounds.so --rounds 1 --calls 2 > $O/r05ac_wdp_bounds_mix.txt 2>&1 || exit 11
timeout -k 10 400 python3 -u tools/replay_study.py --variants shipped,lib=tools/lib/libkarma_crc32c_wdp.so --rounds 7 --calls 20 > $O/r05_replay_walk_put_ab.txt 2>&1 || exit 12
