#!/bin/bash
# round-3 GPU pass g: IPM execution modes A/B (monolithic / per-phase kernels / grouped phases) with per-kernel traffic
set -o pipefail
mkdir -p gpurun_out
TAG=r03g MODES="0 1 2" bash tools/ab_phased.sh > gpurun_out/r03g_ab.log 2>&1 || exit $?
grep -v "^step\|iters percentiles" gpurun_out/r03g_ab.log | tail -n 60
