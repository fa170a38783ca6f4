set -e
mkdir -p gpurun_out/r3t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > gpurun_out/r3t/gpu_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --karma-lib bounds > gpurun_out/r3t/gpu_tests_bounds.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3t/smoke.log 2>&1
echo done
