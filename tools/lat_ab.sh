#!/bin/bash
# batch-1 / small-batch latency of library variants: k_ipm ms of quick_bench steps 1-3
# usage: VARS="prev base" bash tools/lat_ab.sh "1:20:1 1:8:2" > log
R=$PWD
libof() { if [ "$1" = base ]; then echo $R/belief-planning_amd/libbmpc.so; else echo $R/belief-planning_amd/libbmpc_$1.so; fi; }
for cfg in $1; do
  IFS=: read B N NB <<< "$cfg"
  for rep in 1 2; do
    for v in $VARS; do
      BMPC_LIBRARY=$(libof $v) timeout -k 10 120 python tools/quick_bench.py $B $N $NB 2>&1 | grep "^step [123]" | \
        sed "s/^/$v B=$B N=$N NB=$NB rep$rep /" | cut -c1-120 || exit 1
    done
  done
done
