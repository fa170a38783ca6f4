#!/usr/bin/env bash
# tools/trace_series.sh TAG [bench args...] -- per-dispatch durations of a long bench run (kernel trace only).
set -euo pipefail
TAG=$1; shift
REPO=$(pwd); export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$REPO/gpurun_out/ts_$TAG" -o run \
    -- python3 "$REPO/bench.py" --no-cpu-baseline "$@" > "$REPO/gpurun_out/ts_$TAG.log" 2>&1
cd "$REPO"
python3 - "$TAG" <<'PY'
import csv, sys, glob
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/ts_{tag}/**/run_kernel_trace.csv", recursive=True) + glob.glob(f"gpurun_out/ts_{tag}/run_kernel_trace.csv")
rows = [r for r in csv.DictReader(open(f[0])) if "k_units" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(tag, len(d), "dispatches; per 20:", " ".join(f"{sum(d[i:i+20])/len(d[i:i+20]):.0f}" for i in range(0, len(d), 20)))
PY
