#!/bin/bash
# round 5: inlining variants (apply_gt / max_step / scaling inlined into their callers) and the
# forward sweep that forms multipliers and slacks (no tree-solve post-pass) vs the shipped
# build, headline; the fused sweep also on config 3 (N=30 NB=2, 15-rhs coupling solve)
set -o pipefail
VARS="base gtinl msinl scinl fuse" TAG=${1:-r05f}_h QB_ARGS="4096 20 1" bash tools/ab_pmc.sh > gpurun_out/${1:-r05f}_h.log 2>&1 || exit $?
VARS="base fuse" TAG=${1:-r05f}_c3 QB_ARGS="4096 30 2" bash tools/ab_pmc.sh > gpurun_out/${1:-r05f}_c3.log 2>&1 || exit $?
tail -n 12 gpurun_out/${1:-r05f}_h.log; tail -n 5 gpurun_out/${1:-r05f}_c3.log
