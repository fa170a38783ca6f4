# round 5: k_segment_once with the chunk loads issued before the table stores (KARMA_SEGMENT_ONCE=3)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "segment" --karma-lib abbounds --timeout 120 --timeout-method thread > $O/r05i_seg_abbounds.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "segment" --timeout 120 --timeout-method thread > $O/r05i_seg_tests.log 2>&1 || exit 11
timeout -k 10 300 python3 -u tools/segment_once_ab.py --variants 1,3 --sizes 64,16 --json $O/r05_segment_early_ab.json > $O/r05_segment_early_ab.txt 2>&1 || exit 12
