#!/usr/bin/env bash
# tools/pmc_passes.sh TAG [bench args...] -- counter passes over bench.py (one rocprofv3 --pmc per pass).
set -euo pipefail
TAG=${1:-probe}; shift || true
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  # a pass over the per-block counter limits hangs after "error code 38": KILL, and stop there
  timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d "$OUT/pass$i" -o run \
      -- python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline "$@" > "$OUT/pass$i.log" 2>&1 \
      || { echo "pass $i failed: $PASS"; exit 1; }
done
