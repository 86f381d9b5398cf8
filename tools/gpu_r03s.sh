#!/bin/bash
# round-3 pass s: GPU suite, band-QP latency / batch timing, then the driver's bench command and
# its rocprofv3 passes (tools/gpu_r03.sh)
set -o pipefail
tag=${1:-r03s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python tools/qp_bench.py 4096 > gpurun_out/${tag}_qp_bench.log 2>&1 || exit $?
cat gpurun_out/${tag}_qp_bench.log
bash tools/gpu_r03.sh ${tag} notests
