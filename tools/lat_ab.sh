#!/bin/bash
# GPU A/B of library variants on the small-batch (one ego per workgroup) path: seeded outputs
# compared with the first variant (one ego and 64 / 32 egos, N=20 NB=1 and N=8 NB=2), then the
# one-ego k_ipm latency interleaved (tools/quick_bench.py, 4 closed-loop steps, two rounds).
# usage: VARS="base v1" TAG=r05m bash tools/lat_ab.sh
set -o pipefail
o=$PWD/gpurun_out/${TAG:-latab}
mkdir -p $o
R=$PWD
libof() { if [ "$1" = base ]; then echo $R/belief-planning_amd/libbmpc.so; else echo $R/belief-planning_amd/libbmpc_$1.so; fi; }
: > $o/vc.log
for cfg in "1 20 1" "64 20 1" "1 8 2" "32 8 2"; do
  set -- $cfg
  for v in $VARS; do
    BMPC_LIBRARY=$(libof $v) timeout -k 10 120 python tools/variant_check.py $o/vc_${v}_$1_$2_$3.npz $1 $2 $3 >> $o/vc.log 2>&1 || exit $?
  done
done
OUT=$o VARS="$VARS" python - <<'PY' >> $o/vc.log
import os, glob, numpy as np
o = os.environ["OUT"]; vs = os.environ["VARS"].split()
for f in sorted(glob.glob(f"{o}/vc_{vs[0]}_*.npz")):
    a = np.load(f)
    for v in vs[1:]:
        b = np.load(f.replace(f"vc_{vs[0]}_", f"vc_{v}_"))
        same = all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "J", "upred"))
        print(f.split("/")[-1][len(vs[0]) + 4:-4], v, "vs", vs[0], "bit-identical", same, "status agree",
              float(np.mean(a["status"] == b["status"])), "max|dJ|/|J|", float(np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"])))),
              "max|du0|", float(np.max(np.abs(a["upred"][:, 0] - b["upred"][:, 0]))))
PY
: > $o/lat.log
for rep in 1 2; do
  for cfg in "1 20 1" "1 8 2"; do
    for v in $VARS; do
      echo "== $v B N NB = $cfg rep $rep" >> $o/lat.log
      BMPC_LIBRARY=$(libof $v) timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step" | cut -c1-120 >> $o/lat.log || exit $?
    done
  done
done
python - $o/lat.log <<'PY'
import re, sys, collections
cur = None; d = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    m = re.match(r"== (\S+) B N NB = (.*) rep", ln)
    if m: cur = (m.group(1), m.group(2)); continue
    m = re.search(r"step ([123]): .*ipm ([\d.]+) ms", ln)
    if m: d[cur].append(float(m.group(2)))
for k, v in sorted(d.items(), key=lambda t: (t[0][1], t[0][0])):
    print(f"LAT {k[0]:8s} B N NB = {k[1]}: ipm mean {sum(v)/len(v):.2f} ms (steps 1-3, n={len(v)})")
PY
grep "bit-identical" $o/vc.log
