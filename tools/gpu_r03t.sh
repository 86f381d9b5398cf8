#!/bin/bash
# round-3 pass t: GPU suite + band-QP timing (the cached / in-LDS band QP), then IPM modes
# 0 (monolithic k_ipm), 2 (grouped out-of-line phases), 3 (grouped phases all inlined) A/B with traffic
set -o pipefail
tag=${1:-r03t}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python tools/qp_bench.py 4096 > gpurun_out/${tag}_qp_bench.log 2>&1 || exit $?
cat gpurun_out/${tag}_qp_bench.log
TAG=${tag}_modes MODES="0 2 3" PMC="0 3" bash tools/ab_phased.sh > gpurun_out/${tag}_modes.log 2>&1 || { tail -n 20 gpurun_out/${tag}_modes.log; exit 1; }
grep -v "^step\|iters percentiles" gpurun_out/${tag}_modes.log | tail -n 30
