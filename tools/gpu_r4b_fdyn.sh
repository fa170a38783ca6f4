#!/usr/bin/env bash
# Round 4, session 2: the fixed kernel's dynamic tail -- its test and the fixed tests on the
# bounds-checked tools build, then the shipped library against the fdyn3 / fdyn5 builds
# (same process, back to back as the bench runs them).
set -euo pipefail
O=gpurun_out/r4fdyn
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "fixed_dynamic_tail or config2 or fixed or init" --karma-lib abbounds > $O/fdyn_abbounds.log 2>&1
tail -1 $O/fdyn_abbounds.log
LIBS="shipped=karma_amd/lib/libkarma_crc32c.so,fdyn3=tools/lib/libkarma_crc32c_fdyn3.so,fdyn5=tools/lib/libkarma_crc32c_fdyn5.so" \
  timeout -k 10 300 python3 -u tools/fixed_libs_ab.py > $O/fixed_libs_ab.log 2>&1
cat $O/fixed_libs_ab.log
echo done
