#!/bin/bash
# round 5: lane-batch shapes -- tb0 clamped batches (round-5 start), base = tail batches
# (BMPC_TAIL_BATCH=1), tb2 = uniform-shape batches (2).  part 1: headline and config 2
# (1,024 egos); part 2: config 3 and one ego
set -o pipefail
if [ "$1" = 1 ]; then
  VARS="base tb0 tb2" TAG=r05aa_h QB_ARGS="4096 20 1" bash tools/ab_pmc.sh > gpurun_out/r05aa_h.log 2>&1 || exit $?
  VARS="base tb0 tb2" TAG=r05aa_c2 QB_ARGS="1024 20 1" bash tools/ab_pmc.sh > gpurun_out/r05aa_c2.log 2>&1 || exit $?
  for f in h c2; do tail -n 9 gpurun_out/r05aa_$f.log; done
else
  VARS="base tb0 tb2" TAG=r05aa_c3 QB_ARGS="4096 30 2" bash tools/ab_pmc.sh > gpurun_out/r05aa_c3.log 2>&1 || exit $?
  VARS="base tb0 tb2" TAG=r05aa_b1 bash tools/lat_ab.sh > gpurun_out/r05aa_b1.log 2>&1 || exit $?
  tail -n 9 gpurun_out/r05aa_c3.log; grep -E "LAT|bit-identical" gpurun_out/r05aa_b1.log
fi
