#!/bin/bash
# round 6, pass c: the GPU suite (pooled replay agreement, recorded-warm-start S / Fx replays, the
# per-step GPU-vs-host agreement printed); the 2-waves-per-ego k_ipm A/B (libbmpc_w2.so,
# BMPC_IPM_W2=1) against the product k_ipm, interleaved, at 4,096 headline egos and config 3;
# smoke; bench
set -o pipefail
tag=${1:-r06c}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=20 -q -rA --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for round in 1 2; do
  for v in prod w2; do
    if [ $v = w2 ]; then E="BMPC_IPM_W2=1 BMPC_LIBRARY=belief-planning_amd/libbmpc_w2.so"; else E="BMPC_UNUSED=0"; fi
    echo "== round $round $v headline" >> $o/w2_ab.log
    env $E timeout -k 10 200 python -u tools/quick_bench.py 4096 20 1 2>&1 | grep "^step" | cut -c1-160 >> $o/w2_ab.log || exit $?
    echo "== round $round $v config3" >> $o/w2_ab.log
    env $E timeout -k 10 300 python -u tools/quick_bench.py 4096 30 2 2>&1 | grep "^step" | cut -c1-160 >> $o/w2_ab.log || exit $?
  done
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
tail -n 1 $o/bench.log | cut -c1-300
