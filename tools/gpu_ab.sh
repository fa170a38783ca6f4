# A/B of the kernel variants + GPU tests (run via gpurun from the repo root)
set -o pipefail
ROUNDS=6 timeout -k 10 200 python tools/variant_bench.py 0 1 2 6 > gpurun_out/variants.log 2>&1 || { cat gpurun_out/variants.log; exit 1; }
cat gpurun_out/variants.log
for v in 0 1; do
  KARMA_RAGGED_VARIANT=$v timeout -k 10 200 python bench.py --workload ragged --no-cpu-baseline > gpurun_out/bench_ragged_v$v.log 2>&1 || { tail -5 gpurun_out/bench_ragged_v$v.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/bench_ragged_v$v.log').read().strip().splitlines()[-1]);print('ragged v$v', d['value'], d['roofline'])"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
