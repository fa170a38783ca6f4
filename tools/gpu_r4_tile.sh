#!/usr/bin/env bash
# Round 4: byte-grid tile size (2, 4, 8 KiB tools builds) on configs[2] and aligned layouts; the
# isolated segment call's cost split (host enqueue, launch, kernel; rocprofv3 kernel trace of the
# segment A/B); the lifetime test's loop replicated with free memory every 100 streams.
set -euo pipefail
O=gpurun_out/r4tile
mkdir -p $O
GRID_MODES="1 2" timeout -k 10 400 python3 -u tools/ragged_study.py > $O/study_t2048_modes.log 2>&1
cat $O/study_t2048_modes.log
for T in 4096 8192; do
  KARMA_STUDY_LIB=tools/lib/libkarma_crc32c_ab_t$T.so timeout -k 10 300 python3 -u tools/ragged_gap.py --case config3,ragged4k --no-log --calls 10 > $O/gap_t$T.log 2>&1
  cat $O/gap_t$T.log
  KARMA_STUDY_LIB=tools/lib/libkarma_crc32c_ab_t$T.so timeout -k 10 400 python3 -u tools/ragged_study.py > $O/study_t$T.log 2>&1
  cat $O/study_t$T.log
done
timeout -k 10 200 python3 -u tools/call_overhead.py --json $O/call_overhead.json > $O/call_overhead.log 2>&1
cat $O/call_overhead.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_seg -o seg -- python3 -u tools/segment_once_ab.py --sizes 64,1 --rounds 2 > $O/seg_prof.log 2>&1
tail -3 $O/seg_prof.log
timeout -k 10 300 python3 -u tools/lifetime_probe.py 50 > $O/lifetime_probe.log 2>&1
cat $O/lifetime_probe.log
echo done
