#!/bin/bash
# round 5: batched tree-solve post-pass on the headline's coupling solve (rb6 = 4 rhs per pass
# from 6 rhs on, rb6x8 = 8 per pass) vs the shipped threshold (8 rhs), headline and config 3
set -o pipefail
VARS="base rb6 rb6x8" TAG=${1:-r05e}_h QB_ARGS="4096 20 1" bash tools/ab_pmc.sh > gpurun_out/${1:-r05e}_h.log 2>&1 || exit $?
VARS="base rb6 rb6x8" TAG=${1:-r05e}_c3 QB_ARGS="4096 30 2" bash tools/ab_pmc.sh > gpurun_out/${1:-r05e}_c3.log 2>&1 || exit $?
tail -n 8 gpurun_out/${1:-r05e}_h.log gpurun_out/${1:-r05e}_c3.log
