#!/bin/bash
# round-3 GPU pass n: support-restricted cone coupling dots + wider cone groups (fused passes) on NB=2 plans
set -o pipefail
mkdir -p gpurun_out/r03n
for cfg in "4096 20 1" "4096 8 2" "4096 30 2" "1 8 2" "1 30 2"; do
  echo "== $cfg" >> gpurun_out/r03n/lat.log
  timeout -k 10 200 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> gpurun_out/r03n/lat.log || exit $?
done
cat gpurun_out/r03n/lat.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03n/gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03n/gpu_tests.log
