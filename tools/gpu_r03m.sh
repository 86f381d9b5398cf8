#!/bin/bash
# round-3 GPU pass m: GPU suite (small batches of large trees on the multi-wave kernel), phase profiles
set -o pipefail
mkdir -p gpurun_out/r03m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03m/gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03m/gpu_tests.log
P=belief-planning_amd/libbmpc_prof.so
for cfg in "1 8 2" "4096 20 1" "4096 30 2"; do
  echo "== $cfg" >> gpurun_out/r03m/phase.log
  BMPC_LIBRARY=$P timeout -k 10 300 python tools/phase_profile.py $cfg >> gpurun_out/r03m/phase.log 2>&1 || exit $?
done
cat gpurun_out/r03m/phase.log
