#!/bin/bash
# round 5: kkt_solve_pair split so the IPM loop calls the coupling solve and the pair's
# refinement directly (BMPC_FLAT_PAIR=1: scratch stack 2,040 -> 1,544 B/lane), headline + config 3
set -o pipefail
VARS="base flat" TAG=${1:-r05i}_h QB_ARGS="4096 20 1" bash tools/ab_pmc.sh > gpurun_out/${1:-r05i}_h.log 2>&1 || exit $?
VARS="base flat" TAG=${1:-r05i}_c3 QB_ARGS="4096 30 2" bash tools/ab_pmc.sh > gpurun_out/${1:-r05i}_c3.log 2>&1 || exit $?
tail -n 6 gpurun_out/${1:-r05i}_h.log; tail -n 6 gpurun_out/${1:-r05i}_c3.log
