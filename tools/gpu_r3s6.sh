set -e
mkdir -p gpurun_out/r3s
timeout -k 10 300 python3 -u tools/replay_study.py --variants shipped,sub=131072,sub=262144,sub=524288,sub=1048576 --rounds 3 > gpurun_out/r3s/replay_sub2.txt 2>&1
echo done
