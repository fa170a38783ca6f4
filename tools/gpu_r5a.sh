#!/bin/bash
# Round-5 first GPU pass: the group_unit load fix (ragged A/B against the round-4 library), the
# single-segment latency split (C++ loop, Python overhead tool, arrival-fold A/B), the FETCH_SIZE
# calibration on header-shaped reads, then the parity / lifetime / multi-host / WAL tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so,pipe4=tools/lib/libkarma_crc32c_pipe4.so,pipe6=tools/lib/libkarma_crc32c_pipe6.so" \
  timeout -k 10 300 python -u tools/ragged_study.py > $O/r05_ragged_group_fix.txt 2>&1 || exit 11
timeout -k 10 120 tools/bin/segment_loop 64 2000 > $O/r05_segment_loop.json 2>&1 || exit 12
timeout -k 10 120 python -u tools/call_overhead.py > $O/r05_call_overhead.txt 2>&1 || exit 13
timeout -k 10 240 python -u tools/segment_once_ab.py --variants 1,2 --sizes 64,16 > $O/r05_segment_arrive_ab.txt 2>&1 || exit 14
timeout -k 10 120 tools/bin/fetch_calib > $O/r05_fetch_calib.json 2>&1 || exit 15
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/calib -o run -- tools/bin/fetch_calib > $O/r05_fetch_calib_prof.log 2>&1 || exit 16
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifetime.py tests/test_gpu_multi_host.py tests/test_gpu_wal.py -x -q --timeout 300 --timeout-method thread > $O/r05a_gpu_tests.log 2>&1 || exit 17
exit 0
