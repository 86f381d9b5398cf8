#!/bin/bash
# round 6, pass i: one-ego latency of the small-batch kernel on 2 waves per ego (tools build
# libbmpc_b2.so, BMPC_BLOCK_WAVES=2) against the product's 4 waves, interleaved
set -o pipefail
tag=${1:-r06i}
o=gpurun_out/$tag
mkdir -p $o
: > $o/lat.log
for rep in 1 2; do
  for cfg in "1 20 1" "1 8 2"; do
    echo "== base4 B N NB = $cfg rep $rep" >> $o/lat.log
    timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step" | cut -c1-120 >> $o/lat.log || exit $?
    echo "== b2 B N NB = $cfg rep $rep" >> $o/lat.log
    BMPC_BLOCK_WAVES=2 BMPC_LIBRARY=belief-planning_amd/libbmpc_b2.so timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step" | cut -c1-120 >> $o/lat.log || exit $?
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
