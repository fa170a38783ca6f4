set -e
bash tools/profile_all.sh r03
bash tools/pmc_replay.sh r03
echo done
