#!/bin/bash
# round 5: k_tree's register budget (BMPC_TREE_WPE 4 / 3 waves per SIMD vs the compiler's 220
# VGPRs = 2): outputs compared, k_tree time of the headline batch interleaved
set -o pipefail
o=gpurun_out/r05ad
mkdir -p $o
R=$PWD
libof() { if [ "$1" = base ]; then echo $R/belief-planning_amd/libbmpc.so; else echo $R/belief-planning_amd/libbmpc_$1.so; fi; }
for v in base tw4 tw3; do
  BMPC_LIBRARY=$(libof $v) timeout -k 10 150 python tools/variant_check.py $o/vc_$v.npz 4096 20 1 >> $o/vc.log 2>&1 || exit $?
done
python - $o <<'PY' >> $o/vc.log
import sys, numpy as np
o = sys.argv[1]; a = np.load(f"{o}/vc_base.npz")
for v in ("tw4", "tw3"):
    b = np.load(f"{o}/vc_{v}.npz")
    print(v, "bit-identical", all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "J", "upred")))
PY
: > $o/t.log
for rep in 1 2; do for v in base tw4 tw3; do
  echo "== $v" >> $o/t.log
  BMPC_LIBRARY=$(libof $v) timeout -k 10 150 python tools/quick_bench.py 4096 20 1 2>&1 | grep "^step [123]" | cut -c1-100 >> $o/t.log || exit $?
done; done
python - $o/t.log <<'PY'
import re, sys, collections
cur = None; d = collections.defaultdict(list); e = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    m = re.match(r"== (\S+)", ln)
    if m: cur = m.group(1); continue
    m = re.search(r"tree ([\d.]+) ms  ipm ([\d.]+) ms", ln)
    if m: d[cur].append(float(m.group(1))); e[cur].append(float(m.group(2)))
for k in d: print(f"TREE {k}: k_tree mean {sum(d[k])/len(d[k]):.3f} ms, k_ipm {sum(e[k])/len(e[k]):.2f} ms (n={len(d[k])})")
PY
cat $o/vc.log | grep bit-identical
