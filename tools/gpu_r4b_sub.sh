#!/usr/bin/env bash
# Round 4, session 2: the replay walk's sub-range size with direct header rounds (the planner's
# default against smaller and larger sub-ranges), 1M x 180 B and configs[2]'s mix, rotated images.
set -euo pipefail
O=gpurun_out/r4sub
mkdir -p $O
timeout -k 10 300 python3 -u tools/replay_study.py --rounds 5 --variants shipped,sub=12288,sub=16384,sub=24576,sub=32768,sub=65536 > $O/replay_sub_180.log 2>&1
cat $O/replay_sub_180.log
timeout -k 10 300 python3 -u tools/replay_study.py --rounds 5 --size 1000 --count 200000 --variants shipped,sub=16384,sub=24576,sub=65536 > $O/replay_sub_1000.log 2>&1
cat $O/replay_sub_1000.log
timeout -k 10 400 python3 -u tools/replay_study.py --rounds 3 --calls 5 --mix config3 --variants shipped,sub=16384,sub=24576 > $O/replay_sub_mix.log 2>&1
cat $O/replay_sub_mix.log
echo done
