# round 5: fold trees through DPP / readlane (k_segment_once, k_combine_block, the fused fold, WAVE_COMB, wave_tree)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05y_gpu_tests.log 2>&1 || exit 11
timeout -k 10 400 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 8 --libs prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so --json $O/r05_segment_dpp_ab.json > $O/r05_segment_dpp_ab.log 2>&1 || exit 12
CASES="1M x 4 KiB,64 x 64 MiB" LIBS="new=karma_amd/lib/libkarma_crc32c.so,prev=tools/lib/libkarma_crc32c_prev.so" timeout -k 10 400 python3 -u tools/fixed_libs_ab.py > $O/r05_fixed_dpp_ab.txt 2>&1 || exit 14
timeout -k 10 200 python3 bench.py --workload segment > $O/r05_bench_segment_dpp.json 2> $O/r05_bench_segment_dpp.err || exit 13
