set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --workload ragged --no-cpu-baseline > gpurun_out/bench_ragged.log 2>&1 || exit 1
cat gpurun_out/bench_ragged.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_ragged -o run -- python3 $R/bench.py --workload ragged --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/tr_ragged.log 2>&1 || exit 1
cd $R; find gpurun_out/tr_ragged -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
