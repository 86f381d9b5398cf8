#!/bin/bash
# GPU A/B of library variants (libbmpc_<tag>.so; "base" = libbmpc.so): outputs of one seeded
# 4096-ego batch compared with the first variant, interleaved k_ipm timings, optional phase
# profile of the current build (PROFILE=1, libbmpc_prof.so) and the GPU suite (TESTS=1).
# usage: VARS="prev v1 base" TAG=r03d bash tools/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
tag=${TAG:-ab}
SKIP_TESTS=1 VARS="$VARS" timeout -k 10 900 bash tools/ab_fuse.sh > gpurun_out/${tag}_ab.log 2>&1 || exit $?
if [ -n "$PROFILE" ]; then
  BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 300 python tools/phase_profile.py 4096 \
    > gpurun_out/${tag}_phase_profile.log 2>&1 || exit $?
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
  tail -n 2 gpurun_out/${tag}_gpu_tests.log
fi
grep -v "^==\|^step" gpurun_out/${tag}_ab.log | tail -n 12
