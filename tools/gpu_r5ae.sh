# round 5: k_segment_once with its tables from immediates (KARMA_SEGMENT_CT, tools build)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u tools/segment_once_ab.py --sizes 64,16,1 --rounds 8 --variants 1,ct --json $O/r05_segment_ct_ab.json > $O/r05_segment_ct_ab.log 2>&1 || exit 12
