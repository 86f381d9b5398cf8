#!/bin/bash
# round-3 pass v: blocked wave-level band QP -- parity (band-QP / belief-MPC / Highway_env GPU tests),
# single-problem latency and its cycle split (BMPC_BQP_PROF build), batch throughput
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bandqp.py tests/test_predictive_controllers.py tests/test_highway_env_belief.py \
  -m gpu -x -v -rA --timeout 120 --timeout-method thread > gpurun_out/r03v_qp_tests.log 2>&1 || { tail -n 40 gpurun_out/r03v_qp_tests.log; exit 1; }
tail -n 1 gpurun_out/r03v_qp_tests.log
BMPC_LIBRARY=belief-planning_amd/libbmpc_bqpprof.so timeout -k 10 120 python tools/qp_lat.py 3 2>&1 | tail -n 3
timeout -k 10 120 python tools/qp_lat.py 30 > gpurun_out/r03v_qp_lat.log 2>&1 || exit $?
cat gpurun_out/r03v_qp_lat.log
timeout -k 10 300 python tools/qp_bench.py 4096 > gpurun_out/r03v_qp_bench.log 2>&1 || exit $?
cat gpurun_out/r03v_qp_bench.log
