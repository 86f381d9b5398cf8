#!/bin/bash
# GPU-box driver: parity tests, then the bench; stops at the first crash / timeout.
# usage: tools/gpu_run.sh TAG [bench args...]
tag=${1:-r01}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rA > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -3 gpurun_out/${tag}_bench.log
exit $rc2
