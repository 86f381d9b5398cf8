#!/bin/bash
# A/B of a library variant against the committed build on every workload it can touch: one-ego
# latency (tools/lat_ab.sh), seeded-batch bit-identity at 4096 headline egos and config 3, and the
# bench's headline / config-3 throughput interleaved.  usage: A=c1 B=lat6 TAG=r06t bash tools/gpu_r06t.sh
set -o pipefail
A=${A:-c1}; B=${B:-lat6}; tag=${TAG:-r06t}
o=gpurun_out/$tag
mkdir -p $o
libof() { [ "$1" = base ] && echo $PWD/belief-planning_amd/libbmpc.so || echo $PWD/belief-planning_amd/libbmpc_$1.so; }
VARS="$A $B" TAG=$tag timeout -k 10 600 bash tools/lat_ab.sh > $o/lat_ab.out 2>&1 || exit $?
for v in $A $B; do
  BMPC_LIBRARY=$(libof $v) timeout -k 10 150 python tools/variant_check.py $o/vb_${v}_4096_20_1.npz 4096 20 1 >> $o/vb.log 2>&1 || exit $?
  BMPC_LIBRARY=$(libof $v) timeout -k 10 150 python tools/variant_check.py $o/vb_${v}_4096_30_2.npz 4096 30 2 >> $o/vb.log 2>&1 || exit $?
done
python - $o $A $B <<'PY' >> $o/vb.log
import sys, numpy as np
o, a, b = sys.argv[1:]
for cfg in ("4096_20_1", "4096_30_2"):
    x, y = np.load(f"{o}/vb_{a}_{cfg}.npz"), np.load(f"{o}/vb_{b}_{cfg}.npz")
    print(cfg, b, "vs", a, "bit-identical", all(np.array_equal(x[k], y[k]) for k in ("status", "iters", "J", "upred")))
PY
for rep in 1 2; do
  for v in $A $B; do
    echo "== $v headline rep $rep" >> $o/bench.log
    BMPC_LIBRARY=$(libof $v) timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -n 1 | cut -c1-200 >> $o/bench.log || exit $?
    echo "== $v config3 rep $rep" >> $o/bench.log
    BMPC_LIBRARY=$(libof $v) timeout -k 10 300 python bench.py --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | tail -n 1 | cut -c1-200 >> $o/bench.log || exit $?
  done
done
tail -n 4 $o/lat_ab.out; cat $o/vb.log | grep bit-identical; cat $o/bench.log
