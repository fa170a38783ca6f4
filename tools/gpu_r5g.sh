# round 5: full GPU suite on the current tree, ragged A/B against the round's start, the bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r05g_gpu_tests.log 2>&1 || exit 10
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05g_ragged.txt 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $O/r05g_bench.json 2> $O/r05g_bench.err || exit 12
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 50 --warmup 10 > $O/r05g_bench_ragged.json 2> $O/r05g_bench_ragged.err || exit 13
