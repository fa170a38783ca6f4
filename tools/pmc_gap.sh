#!/usr/bin/env bash
# tools/pmc_gap.sh TAG CASES -- rocprofv3 counter passes over tools/ragged_gap.py, one process
# per (case, pass), each under its own time limit (run from the repo root on the GPU box).
# Summarise with: python tools/pmc_kernels.py gpurun_out/pmc_gap_TAG/<case> out.json k_units_
set -euo pipefail
TAG=${1:-probe}
CASES=${2:-"fixed_v1 ragged4k config3"}
REPO=$(pwd)
export TMPDIR=/tmp
for C in $CASES; do
  OUT=$REPO/gpurun_out/pmc_gap_$TAG/$C
  mkdir -p "$OUT"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
      -- python3 "$REPO/tools/ragged_gap.py" --case "$C" --calls 5 --no-log > "$OUT/trace.log" 2>&1 \
      || { echo "trace failed: $C"; exit 1; }
  i=0
  for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
              "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d "$OUT/pass$i" -o run \
        -- python3 "$REPO/tools/ragged_gap.py" --case "$C" --calls 5 --no-log > "$OUT/pass$i.log" 2>&1 \
        || { echo "pass $i failed: $C $PASS"; exit 1; }
  done
  cd "$REPO"
done
echo done
