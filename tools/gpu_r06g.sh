#!/bin/bash
# round 6, pass g: the fused closed loop (bmpc_loop_device / k_loop): its bit-identity test, then
# bench.py --loop fused vs --loop steps interleaved (3 rounds), then the GPU suite
set -o pipefail
tag=${1:-r06g}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_loop_gpu.py -x -v -rA --timeout 240 --timeout-method thread > $o/loop_test.log 2>&1 || exit $?
for r in 1 2 3; do
  for m in steps fused; do
    echo "== round $r $m" >> $o/loop_ab.log
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --loop $m 2>&1 | tail -n 1 | cut -c1-220 >> $o/loop_ab.log || exit $?
  done
done
timeout -k 10 300 python bench.py --gpus 1 --N 30 --NB 2 --steps 5 --warmup 2 --no-cpu-baseline --loop steps 2>&1 | tail -n 1 | cut -c1-220 >> $o/loop_ab.log || exit $?
timeout -k 10 300 python bench.py --gpus 1 --N 30 --NB 2 --steps 5 --warmup 2 --no-cpu-baseline --loop fused 2>&1 | tail -n 1 | cut -c1-220 >> $o/loop_ab.log || exit $?
true
true
cat $o/loop_ab.log
