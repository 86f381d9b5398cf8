#!/bin/bash
# round-3 GPU pass p: quad-per-branch Riccati (no scratch in the recursion)
set -o pipefail
mkdir -p gpurun_out/r03p
for cfg in "4096 20 1" "4096 8 2" "4096 30 2" "1 8 2"; do
  for m in 0 2; do
    [ "$m" = 2 ] && [ "$cfg" != "4096 20 1" ] && continue
    echo "== mode $m $cfg" >> gpurun_out/r03p/lat.log
    BMPC_IPM_PHASED=$m timeout -k 10 200 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> gpurun_out/r03p/lat.log || exit $?
  done
done
cat gpurun_out/r03p/lat.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03p/gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03p/gpu_tests.log
