#!/bin/bash
# round 6, pass d: wave reductions on DPP / permlane swaps (product, BMPC_DPP_REDUCE=1) against the
# ds_bpermute butterflies (libbmpc_shfl.so): bit-identity + one-ego latency (lat_ab.sh), headline
# and config-3 k_ipm time + PMC bytes (ab_pmc.sh); then the GPU suite, smoke, bench
set -o pipefail
tag=${1:-r06d}
VARS="shfl base" TAG=${tag}_lat timeout -k 10 600 bash tools/lat_ab.sh > gpurun_out/${tag}_lat.log 2>&1 || exit $?
VARS="shfl base" TAG=${tag}_ab QB_ARGS="4096 20 1" timeout -k 10 900 bash tools/ab_pmc.sh > gpurun_out/${tag}_ab.log 2>&1 || exit $?
VARS="shfl base" TAG=${tag}_ab3 QB_ARGS="4096 30 2" timeout -k 10 900 bash tools/ab_pmc.sh > gpurun_out/${tag}_ab3.log 2>&1 || exit $?
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=20 -q -rA --timeout 300 --timeout-method thread > gpurun_out/$tag/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$tag/bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/$tag/bench.log | cut -c1-300
