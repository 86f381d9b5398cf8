#!/bin/bash
# GPU A/B of the IPM execution modes of one library (BMPC_IPM_PHASED = 0: monolithic k_ipm,
# 1: one kernel per phase, 2: one kernel calling grouped phase functions): outputs of one seeded
# 4096-ego batch compared with mode 0, interleaved timings, a rocprofv3 kernel trace of mode 1
# (per-phase kernel times) and FETCH_SIZE / WRITE_SIZE of every mode (per phase for mode 1).
# usage: TAG=r03f MODES="0 1 2 1s4" bash tools/ab_phased.sh   (MsN: mode M with BMPC_PH_STREAMS=N)
# the modes live in a tools-only build: python tools/build_variant.py ph -DBMPC_WITH_PHASED, then
# BMPC_LIBRARY=$PWD/belief-planning_amd/libbmpc_ph.so
set -o pipefail
tag=${TAG:-abph}
modes=${MODES:-0 1 2}
# run "MsN" -> BMPC_IPM_PHASED=M BMPC_PH_STREAMS=N
envof() { local m=$1; if [[ $m == *s* ]]; then echo "BMPC_IPM_PHASED=${m%s*} BMPC_PH_STREAMS=${m#*s}"; else echo "BMPC_IPM_PHASED=$m BMPC_PH_STREAMS=1"; fi; }
out=gpurun_out/$tag
mkdir -p $out
for v in $modes; do
  env $(envof $v) timeout -k 10 150 python tools/variant_check.py $out/vc_$v.npz 4096 || exit $?
done
MODES="$modes" python - $out <<'PY' || exit $?
import os, sys
import numpy as np
a = np.load(sys.argv[1] + "/vc_0.npz")
for m in os.environ["MODES"].split()[1:]:
    b = np.load(sys.argv[1] + f"/vc_{m}.npz")
    print(f"mode {m} vs 0:", {k: bool(np.array_equal(a[k], b[k])) for k in a.files},
          "max |dJ|/|J| %.3e" % np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"]))),
          "status agree %.4f" % np.mean(a["status"] == b["status"]), "iters mean %.2f -> %.2f" % (a["iters"].mean(), b["iters"].mean()))
PY
: > $out/ab.log
for r in 1 2; do
  for v in $modes; do
    echo "== mode=$v run $r" >> $out/ab.log
    env $(envof $v) timeout -k 10 200 python tools/quick_bench.py 4096 2>&1 | grep "^step [123]" | cut -c1-130 >> $out/ab.log || exit $?
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
if [ -n "$TRACE" ]; then
  (cd /tmp && export TMPDIR=/tmp && export $(envof $TRACE) && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run \
     --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/quick_bench.py 4096 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1) || exit $?
  python3 tools/ph_kernel_summary.py $out/prof > $out/ph_kernels.txt || exit $?
  cat $out/ph_kernels.txt
fi
pmc=${PMC-$modes}   # modes whose FETCH_SIZE / WRITE_SIZE passes run (PMC="" for none)
[ -z "$pmc" ] && exit 0
for v in $pmc; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && export $(envof $v) && timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $GRAFT_REPO_ROOT/$out/pmc_${v}_$c \
       -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/quick_bench.py 4096 > $GRAFT_REPO_ROOT/$out/pmc_${v}_$c.log 2>&1) || exit $?
  done
done
python3 tools/ph_pmc_summary.py $out $pmc > $out/pmc.txt || exit $?
cat $out/pmc.txt
