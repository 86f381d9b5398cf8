#!/bin/bash
# one-ego k_ipm latency of the plain highway plan against the BMPC_PLAN_TRANSFORM plan that the
# drop-in BranchMPC_CVaR creates (per-ego S / Fx / bx path), interleaved, two reps
# usage: bash tools/lat_xform.sh "1 8 2" "1 20 1" > log
for rep in 1 2; do
  for cfg in "$@"; do
    for t in "" 1; do
      echo "== transform=[${t:-0}] cfg $cfg rep $rep"
      QB_TRANSFORM=$t timeout -k 10 100 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" || exit 1
    done
  done
done
