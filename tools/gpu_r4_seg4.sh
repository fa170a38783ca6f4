#!/usr/bin/env bash
# Round 4: where the one-segment kernel's first 10 us go (stamps after the table and chunk load
# issue; a second, warm back-to-back call logged too).
set -euo pipefail
O=gpurun_out/r4seg4
mkdir -p $O
timeout -k 10 200 python3 -u tools/segment_once_ab.py --sizes 64,1 --rounds 1 --json $O/segment_once_ab.json > $O/segment_once_ab.log 2>&1
cat $O/segment_once_ab.log
echo done
