#!/bin/bash
# Round-5 second GPU pass: SQ counters of the fixed and ragged units kernels on identical aligned
# 1M x 4 KiB records, the 64 MiB burst probe (item 3), the depth-2 staged
# replay kernel (item 2), the ragged host path's two-stream overlap (item 5) and the append from a
# page-locked image (item 8).
set -o pipefail
export TMPDIR=/tmp
REPO="$GRAFT_REPO_ROOT"
cd "$REPO" || exit 1
O=$REPO/gpurun_out
mkdir -p $O
SHIP=$REPO/karma_amd/lib/libkarma_crc32c.so
AB=$REPO/tools/lib/libkarma_crc32c_ab.so
# the depth-2 staged kernel's first runs: bounds-checked tools build, against the model
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py -k depth2 -x -q --karma-lib abbounds --timeout 120 \
    --timeout-method thread > $O/r05_depth2_abbounds.log 2>&1 || exit 10
timeout -k 10 120 tools/bin/burst_probe > $O/r05_burst_probe.json 2>&1 || exit 11
for C in fixed ragged4k fixed_k1; do
  LIB=$SHIP; [ "$C" = fixed_k1 ] && LIB=$AB
  D=$O/r05_sq_$C
  mkdir -p $D
  cd /tmp
  KARMA_STUDY_LIB=$LIB timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run \
      -- python3 $REPO/tools/ragged_gap.py --case $C --calls 5 --no-log > $D/trace.log 2>&1 || exit 12
  i=0
  for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
              "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
              "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    KARMA_STUDY_LIB=$LIB timeout -s KILL 150 rocprofv3 --pmc $PASS --output-format csv -d $D/pass$i -o run \
        -- python3 $REPO/tools/ragged_gap.py --case $C --calls 5 --no-log > $D/pass$i.log 2>&1 || { echo "pass $i $C failed"; }
  done
  cd $REPO
done
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,ab,ab:KARMA_STAGE_DEPTH=2 --rounds 5 > $O/r05_replay_depth2.txt 2>&1 || exit 13
LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" timeout -k 10 300 python3 -u tools/host_ragged_rate.py --rounds 3 > $O/r05_host_ragged.json 2>&1 || exit 14
timeout -k 10 300 python3 -u bench.py --workload wal_append --steps 10 --warmup 2 > $O/r05_bench_wal_append.json 2>&1 || exit 15
exit 0
