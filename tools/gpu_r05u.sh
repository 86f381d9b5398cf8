#!/bin/bash
# round 5: one-ego latency by launch shape: 4 / 8 waves per ego (BMPC_BLOCK_WAVES) and the
# one-wave k_ipm (BMPC_BLOCK_EGOS=0), N=20 NB=1 and N=8 NB=2, interleaved twice
set -o pipefail
o=gpurun_out/${1:-r05u}
mkdir -p $o
: > $o/lat.log
for rep in 1 2; do
  for cfg in "1 20 1" "1 8 2"; do
    for v in "BMPC_BLOCK_WAVES=4" "BMPC_BLOCK_WAVES=8" "BMPC_BLOCK_EGOS=0"; do
      echo "== $v B N NB = $cfg rep $rep" >> $o/lat.log
      env $v timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step" | cut -c1-120 >> $o/lat.log || exit $?
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
    print(f"LAT {k[0]:20s} B N NB = {k[1]}: ipm mean {sum(v)/len(v):.2f} ms (steps 1-3, n={len(v)})")
PY
