#!/usr/bin/env bash
# tools/pmc_small.sh TAG -- kernel trace + SQ counter passes over the small-record CRC kernels
# (tools/direct_study.py: the 4-lane k_ragged_direct4 and the LDS-staged k_ragged_staged_pipe on
# 1M x 180 B payloads); run via gpurun from the repo root.  One rocprofv3 --pmc per pass.
set -euo pipefail
TAG=${1:-r03}
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_small_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
CMD=(python3 "$REPO/tools/direct_study.py" --variants 0,20 --rounds 1 --calls 5)
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${CMD[@]}" \
    > "$OUT/trace.log" 2>&1
i=0
for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d "$OUT/pass$i" -o run -- "${CMD[@]}" \
      > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed: $PASS"; exit 1; }
done
echo done
