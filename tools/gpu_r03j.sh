#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
TAG=r03j LIBS="prev base" MODES="0 2" bash tools/ab_libs.sh > gpurun_out/r03j_ab.log 2>&1 || exit $?
grep -v "^step\|iters percentiles" gpurun_out/r03j_ab.log | tail -n 30
TAG=r03j8 LIBS="prev base" MODES="0" QB_ARGS="8 2" bash tools/ab_libs.sh > gpurun_out/r03j8_ab.log 2>&1 || exit $?
grep MEAN gpurun_out/r03j8_ab.log
TAG=r03j30 LIBS="prev base" MODES="0" QB_ARGS="30 2" bash tools/ab_libs.sh > gpurun_out/r03j30_ab.log 2>&1 || exit $?
grep MEAN gpurun_out/r03j30_ab.log
