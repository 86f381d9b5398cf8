#!/bin/bash
# round-3 GPU pass f: calibration microbenchmarks, phased-vs-monolithic IPM A/B, GPU suite
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_calib.sh r03f_calib > gpurun_out/r03f_calib.log 2>&1 || exit $?
head -n 4 gpurun_out/r03f_calib.log
TAG=r03f bash tools/ab_phased.sh > gpurun_out/r03f_ab.log 2>&1 || exit $?
cat gpurun_out/r03f_ab.log | grep -v "^step\|iters percentiles" | tail -n 40
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03f_gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03f_gpu_tests.log
