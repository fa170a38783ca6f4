set -e
mkdir -p gpurun_out/r3s
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/r3s/prof_bench" -o run -- python3 "$REPO/bench.py" --steps 50 --warmup 10 --no-cpu-baseline > "$REPO/gpurun_out/r3s/prof_bench.json" 2> "$REPO/gpurun_out/r3s/prof_bench.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/r3s/prof_replay" -o run -- python3 "$REPO/tools/replay_study.py" --variants shipped --rounds 1 --calls 10 > "$REPO/gpurun_out/r3s/prof_replay.log" 2>&1
echo done
