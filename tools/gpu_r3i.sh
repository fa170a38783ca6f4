set -e
mkdir -p gpurun_out/r3i
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 300 python3 -u bench.py --workload ragged --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r3i/ragged.json 2> gpurun_out/r3i/ragged.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/r3i/trace_ragged" -o run -- python3 "$REPO/bench.py" --workload ragged --steps 100 --warmup 20 --no-cpu-baseline > "$REPO/gpurun_out/r3i/trace_ragged.log" 2>&1
cd "$REPO"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ragged" > gpurun_out/r3i/ragged_tests.log 2>&1
echo done
