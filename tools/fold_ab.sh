set -e
for i in 1 2 3; do
  for k in 1 2; do
    KARMA_FOLD_MAX_K=$k timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/fb_${k}_${i}.json 2> gpurun_out/fb_${k}_${i}.err
    python -c "import json,sys; d=json.load(open('gpurun_out/fb_${k}_${i}.json')); print('k=$k run $i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
