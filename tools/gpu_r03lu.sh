#!/bin/bash
# round-3 pass lu: the coupling LU with its trailing update dealt over all lanes (batched loads)
# against the previous commit: headline batch, config 3, one ego N=8 NB=2
set -o pipefail
mkdir -p gpurun_out
TAG=r03lu20 LIBS="prev base" MODES="0" bash tools/ab_libs.sh > gpurun_out/r03lu20_ab.log 2>&1 || { tail -n 20 gpurun_out/r03lu20_ab.log; exit 1; }
grep "vs\|MEAN" gpurun_out/r03lu20_ab.log
TAG=r03lu30 LIBS="prev base" MODES="0" QB_ARGS="30 2" bash tools/ab_libs.sh > gpurun_out/r03lu30_ab.log 2>&1 || { tail -n 20 gpurun_out/r03lu30_ab.log; exit 1; }
grep "vs\|MEAN" gpurun_out/r03lu30_ab.log
TAG=r03lu1 BATCH=1 LIBS="prev base" MODES="0" QB_ARGS="8 2" bash tools/ab_libs.sh > gpurun_out/r03lu1_ab.log 2>&1 || { tail -n 20 gpurun_out/r03lu1_ab.log; exit 1; }
grep "vs\|MEAN" gpurun_out/r03lu1_ab.log
