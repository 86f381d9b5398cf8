#!/bin/bash
# round 5: lane batches without clamped duplicate loads (BMPC_TAIL_BATCH=1: full batches, then
# halving batches for a lane's remainder) vs the shipped clamped batches: headline + config 3
# (k_ipm time + PMC bytes, outputs compared), then the one-ego path; and the LDS-span GPU test
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_blk_lds_gpu.py -v -rA --timeout 300 --timeout-method thread > gpurun_out/r05x_blk_lds_test.log 2>&1 || exit $?
VARS="base tb" TAG=r05y_h QB_ARGS="4096 20 1" bash tools/ab_pmc.sh > gpurun_out/r05y_h.log 2>&1 || exit $?
VARS="base tb" TAG=r05y_c3 QB_ARGS="4096 30 2" bash tools/ab_pmc.sh > gpurun_out/r05y_c3.log 2>&1 || exit $?
VARS="base tb" TAG=r05y_b1 bash tools/lat_ab.sh > gpurun_out/r05y_b1.log 2>&1 || exit $?
tail -n 3 gpurun_out/r05x_blk_lds_test.log; tail -n 6 gpurun_out/r05y_h.log; tail -n 6 gpurun_out/r05y_c3.log; tail -n 8 gpurun_out/r05y_b1.log
