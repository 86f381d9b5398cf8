#!/bin/bash
# round-3 GPU pass k: phase profiles (headline, config 3, config 1), occupancy knob, GPU suite on mode 2
set -o pipefail
mkdir -p gpurun_out
P=belief-planning_amd/libbmpc_prof.so
for cfg in "4096 20 1" "4096 30 2" "1 8 2" "64 8 2"; do
  echo "== $cfg" >> gpurun_out/r03k_phase.log
  BMPC_LIBRARY=$P timeout -k 10 300 python tools/phase_profile.py $cfg >> gpurun_out/r03k_phase.log 2>&1 || exit $?
done
cat gpurun_out/r03k_phase.log
for lds in 0 20000 14000; do
  echo "== lds $lds" >> gpurun_out/r03k_occ.log
  BMPC_IPM_LDS_BYTES=$lds timeout -k 10 200 python tools/quick_bench.py 4096 2>&1 | grep "^step [123]" | cut -c1-100 >> gpurun_out/r03k_occ.log || exit $?
done
cat gpurun_out/r03k_occ.log
BMPC_IPM_PHASED=2 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03k_gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03k_gpu_tests.log
