# round 5: the plan's edge loads with the offsets (ab) or after the scan (pe1)
set -o pipefail
O=gpurun_out
mkdir -p $O
for v in ab pe1; do
  timeout -k 10 300 python3 -u tools/plan_phases.py --lib tools/lib/libkarma_crc32c_$v.so --calls 3 --json $O/r05_plan_phases_$v.json > $O/r05_plan_phases_$v.log 2>&1 || exit 11
done
LIBS="ab=tools/lib/libkarma_crc32c_ab.so,pe1=tools/lib/libkarma_crc32c_pe1.so" timeout -k 10 400 python3 -u tools/ragged_study.py > $O/r05_plan_edges_ab.txt 2>&1 || exit 12
