#!/bin/bash
# round-3 final pass: GPU suite, band-QP latency, the driver's bench command and its rocprofv3 passes
set -o pipefail
tag=${1:-r03fin}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 120 python tools/qp_lat.py 30 > gpurun_out/${tag}_qp_lat.log 2>&1 || exit $?
cat gpurun_out/${tag}_qp_lat.log
bash tools/gpu_r03.sh ${tag} notests
