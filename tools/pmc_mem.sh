#!/usr/bin/env bash
# tools/pmc_mem.sh TAG "case[@lib] ..." -- memory-side counter passes (L2 requests to the fabric, L2
# hits, vector-cache stalls, wave waits) over tools/ragged_gap.py, one process per (case, pass), each
# under its own time limit (run from the repo root on the GPU box).
# Summarise with: python tools/pmc_kernels.py gpurun_out/pmc_mem_TAG/<case> out.json k_units_
set -euo pipefail
TAG=${1:-probe}
CASES=${2:-"fixed ragged4k"}
REPO=$(pwd)
export TMPDIR=/tmp
for CL in $CASES; do
  C=${CL%%@*}
  LIBARG=()
  if [[ "$CL" == *@* ]]; then LIBARG=(--lib "$REPO/${CL#*@}"); fi
  NAME=$C
  if [[ "$CL" == *@* ]]; then NAME=$C$(basename "${CL#*@}" .so | sed 's/libkarma_crc32c//'); fi
  OUT=$REPO/gpurun_out/pmc_mem_$TAG/$NAME
  mkdir -p "$OUT"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
      -- python3 "$REPO/tools/ragged_gap.py" --case "$C" --calls 5 --no-log "${LIBARG[@]}" > "$OUT/trace.log" 2>&1 \
      || { echo "trace failed: $CL"; exit 1; }
  i=0
  for PASS in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
              "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $PASS --output-format csv -d "$OUT/pass$i" -o run \
        -- python3 "$REPO/tools/ragged_gap.py" --case "$C" --calls 5 --no-log "${LIBARG[@]}" > "$OUT/pass$i.log" 2>&1 \
        || { echo "pass $i failed: $CL $PASS"; exit 1; }
  done
  cd "$REPO"
done
echo done
