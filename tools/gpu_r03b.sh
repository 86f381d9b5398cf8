#!/bin/bash
# Round-3 GPU pass: new parity tests first, then the whole GPU suite, the phase-counter profile
# at the metric batch and the default bench.
# usage: bash tools/gpu_r03b.sh TAG
set -o pipefail
tag=${1:-r03b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_xform.py tests/test_config5_gpu.py -m gpu -x -v -rA --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_new_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 300 python tools/phase_profile.py 4096 \
  > gpurun_out/${tag}_phase_profile.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/${tag}_bench.log | cut -c1-300
echo done
