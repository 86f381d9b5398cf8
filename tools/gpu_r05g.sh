#!/bin/bash
# round 5: the GPU parity suite with this round's bars on the current source, smoke(), the bench
set -o pipefail
tag=${1:-r05g}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -rA --timeout 600 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc   # assertion failures (1) go on; faults / timeouts stop here
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
tail -n 3 $o/gpu_tests.log; tail -n 1 $o/bench.log | cut -c1-300
