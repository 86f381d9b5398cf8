#!/bin/bash
# GPU A/B of library builds x IPM modes: one seeded 4096-ego batch through each (outputs compared
# with the first), then interleaved quick_bench timings.
# usage: TAG=r03i LIBS="prev base" MODES="0 2" bash tools/ab_libs.sh   (base = libbmpc.so)
set -o pipefail
tag=${TAG:-ablib}
libs=${LIBS:-prev base}
modes=${MODES:-0}
B=${BATCH:-4096}
out=gpurun_out/$tag
mkdir -p $out
libof() { [ "$1" = base ] && echo belief-planning_amd/libbmpc.so || echo belief-planning_amd/libbmpc_$1.so; }
vars=""
for l in $libs; do for m in $modes; do vars="$vars $l:$m"; done; done
for v in $vars; do
  BMPC_LIBRARY=$(libof ${v%:*}) BMPC_IPM_PHASED=${v#*:} timeout -k 10 150 python tools/variant_check.py $out/vc_${v/:/_}.npz $B || exit $?
done
VARS="$vars" python - $out <<'PY' || exit $?
import os, sys
import numpy as np
vs = os.environ["VARS"].split()
a = np.load(sys.argv[1] + "/vc_%s.npz" % vs[0].replace(":", "_"))
for v in vs[1:]:
    b = np.load(sys.argv[1] + "/vc_%s.npz" % v.replace(":", "_"))
    print(f"{v} vs {vs[0]}:", {k: bool(np.array_equal(a[k], b[k])) for k in a.files},
          "max |dJ|/|J| %.3e" % np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"]))),
          "status agree %.4f" % np.mean(a["status"] == b["status"]),
          "iters mean %.2f -> %.2f" % (a["iters"].mean(), b["iters"].mean()))
PY
: > $out/ab.log
for r in 1 2; do
  for v in $vars; do
    echo "== $v run $r" >> $out/ab.log
    BMPC_LIBRARY=$(libof ${v%:*}) BMPC_IPM_PHASED=${v#*:} timeout -k 10 200 python tools/quick_bench.py $B ${QB_ARGS:-} 2>&1 \
      | grep "^step [123]" | cut -c1-130 >> $out/ab.log || exit $?
  done
done
python - $out/ab.log <<'PY'
import re, sys, collections
d = collections.defaultdict(list); cur = None
for ln in open(sys.argv[1]):
    m = re.match(r"== (\S+) run", ln)
    if m: cur = m.group(1); continue
    m = re.search(r"ipm ([\d.]+) ms", ln)
    if m: d[cur].append(float(m.group(1)))
with open(sys.argv[1], "a") as f:
    for k, v in d.items():
        f.write(f"MEAN {k}: {sum(v)/len(v):.3f} ms over {len(v)}\n")
PY
grep MEAN $out/ab.log
