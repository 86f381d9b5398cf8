#!/bin/bash
# GPU A/B of the phase-per-kernel IPM against the monolithic k_ipm (same library, BMPC_IPM_PHASED
# = 1 / 0): outputs of one seeded 4096-ego batch compared bit for bit, interleaved timings, a
# rocprofv3 kernel trace of the phased solves (per-phase kernel times), the bench line.
# usage: TAG=r03f bash tools/ab_phased.sh
set -o pipefail
tag=${TAG:-abph}
out=gpurun_out/$tag
mkdir -p $out
for v in 0 1; do
  BMPC_IPM_PHASED=$v timeout -k 10 150 python tools/variant_check.py $out/vc_$v.npz 4096 || exit $?
done
python - $out <<'PY' || exit $?
import sys
import numpy as np
a, b = np.load(sys.argv[1] + "/vc_0.npz"), np.load(sys.argv[1] + "/vc_1.npz")
print("phased vs monolithic:", {k: bool(np.array_equal(a[k], b[k])) for k in a.files},
      "max |dJ| %.3e" % np.max(np.abs(a["J"] - b["J"])), "status agree %.4f" % np.mean(a["status"] == b["status"]))
PY
: > $out/ab.log
for r in 1 2; do
  for v in 0 1; do
    echo "== phased=$v run $r" >> $out/ab.log
    BMPC_IPM_PHASED=$v timeout -k 10 200 python tools/quick_bench.py 4096 2>&1 | grep "^step [123]" | cut -c1-130 >> $out/ab.log || exit $?
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
(cd /tmp && export TMPDIR=/tmp && BMPC_IPM_PHASED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run \
   --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/quick_bench.py 4096 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1) || exit $?
python3 tools/ph_kernel_summary.py $out/prof > $out/ph_kernels.txt || exit $?
cat $out/ph_kernels.txt
BMPC_IPM_PHASED=1 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.log 2>&1 || exit $?
tail -n 1 $out/bench.log | cut -c1-300
