#!/bin/bash
# round-3 GPU pass h: phase-per-kernel IPM on 1 / 2 / 4 / 8 sub-batch streams vs monolithic and grouped
set -o pipefail
mkdir -p gpurun_out
TAG=r03h MODES="0 1s1 1s2 1s4 1s8 2" PMC="1s4" TRACE=1s4 bash tools/ab_phased.sh > gpurun_out/r03h_ab.log 2>&1 || exit $?
grep -v "^step\|iters percentiles" gpurun_out/r03h_ab.log | tail -n 60
