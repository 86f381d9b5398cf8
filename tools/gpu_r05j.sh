#!/bin/bash
# round 5: kkt_refine_pair's correction back halves as calls of their own (BMPC_REFINE_CALLS=1:
# scratch stack 1,544 -> 1,440 B/lane) vs the shipped flat-pair build, headline + config 3
set -o pipefail
VARS="base rcall" TAG=${1:-r05j}_h QB_ARGS="4096 20 1" bash tools/ab_pmc.sh > gpurun_out/${1:-r05j}_h.log 2>&1 || exit $?
VARS="base rcall" TAG=${1:-r05j}_c3 QB_ARGS="4096 30 2" bash tools/ab_pmc.sh > gpurun_out/${1:-r05j}_c3.log 2>&1 || exit $?
tail -n 6 gpurun_out/${1:-r05j}_h.log; tail -n 6 gpurun_out/${1:-r05j}_c3.log
