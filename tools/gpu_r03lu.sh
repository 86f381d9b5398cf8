#!/bin/bash
# round-3 pass cv (was lu): the coupling LU with its trailing update dealt over all lanes, pivots and rhs in LDS
# against the previous commit: headline batch, config 3, one ego N=8 NB=2
set -o pipefail
mkdir -p gpurun_out
TAG=r03rw20 LIBS="prev base" MODES="0" bash tools/ab_libs.sh > gpurun_out/r03rw20_ab.log 2>&1 || { tail -n 20 gpurun_out/r03rw20_ab.log; exit 1; }
grep "vs\|MEAN" gpurun_out/r03rw20_ab.log
TAG=r03rw30 LIBS="prev base" MODES="0" QB_ARGS="30 2" bash tools/ab_libs.sh > gpurun_out/r03rw30_ab.log 2>&1 || { tail -n 20 gpurun_out/r03rw30_ab.log; exit 1; }
grep "vs\|MEAN" gpurun_out/r03rw30_ab.log
TAG=r03rw1 BATCH=1 LIBS="prev base" MODES="0" QB_ARGS="8 2" bash tools/ab_libs.sh > gpurun_out/r03rw1_ab.log 2>&1 || { tail -n 20 gpurun_out/r03rw1_ab.log; exit 1; }
grep "vs\|MEAN" gpurun_out/r03rw1_ab.log
