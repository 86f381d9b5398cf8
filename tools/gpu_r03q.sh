#!/bin/bash
# round-3 GPU pass q: A/B quad Riccati (base) vs HEAD (prev), headline and config 3, modes 0/2
set -o pipefail
mkdir -p gpurun_out
TAG=r03q LIBS="prev base" MODES="0 2" bash tools/ab_libs.sh > gpurun_out/r03q_ab.log 2>&1 || exit $?
grep -v "^step\|iters percentiles" gpurun_out/r03q_ab.log | tail -n 12
TAG=r03q30 LIBS="prev base" MODES="0" QB_ARGS="30 2" bash tools/ab_libs.sh > gpurun_out/r03q30_ab.log 2>&1 || exit $?
grep MEAN gpurun_out/r03q30_ab.log
