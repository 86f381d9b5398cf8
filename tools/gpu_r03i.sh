#!/bin/bash
# round-3 GPU pass i: tree solve with the slack passes folded into the sweeps + Woodbury column skipping (A/B vs prev)
set -o pipefail
mkdir -p gpurun_out
TAG=r03i LIBS="prev base" MODES="0 2" bash tools/ab_libs.sh > gpurun_out/r03i_ab.log 2>&1 || exit $?
grep -v "^step\|iters percentiles" gpurun_out/r03i_ab.log | tail -n 30
TAG=r03i8 LIBS="prev base" MODES="0" QB_ARGS="8 2" BATCH=4096 bash tools/ab_libs.sh > gpurun_out/r03i8_ab.log 2>&1 || exit $?
grep MEAN gpurun_out/r03i8_ab.log
