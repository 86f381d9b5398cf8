#!/bin/bash
# round-3 GPU pass o: phase profiles after the coupling changes; the driver's bench command
set -o pipefail
mkdir -p gpurun_out/r03o
P=belief-planning_amd/libbmpc_prof.so
for cfg in "4096 20 1" "4096 30 2" "1 8 2"; do
  echo "== $cfg" >> gpurun_out/r03o/phase.log
  BMPC_LIBRARY=$P timeout -k 10 300 python tools/phase_profile.py $cfg >> gpurun_out/r03o/phase.log 2>&1 || exit $?
done
cat gpurun_out/r03o/phase.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03o/bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/r03o/bench.log | cut -c1-400
