#!/bin/bash
# GPU A/B of library variants (libbmpc_<tag>.so; "base" = libbmpc.so) on one seeded 4096-ego
# highway batch: outputs compared with the first variant, interleaved k_ipm timings (HIP
# events), then per-dispatch FETCH_SIZE / WRITE_SIZE of k_ipm from separate rocprofv3 passes.
# usage: VARS="base v1" TAG=r04a [QB_ARGS="4096 20 1"] bash tools/ab_pmc.sh
set -o pipefail
tag=${TAG:-ab}
VARS=${VARS:-base}
QB=${QB_ARGS:-4096}
R=$PWD
out=$R/gpurun_out/$tag
mkdir -p $out
libof() { if [ "$1" = base ]; then echo $R/belief-planning_amd/libbmpc.so; else echo $R/belief-planning_amd/libbmpc_$1.so; fi; }
for v in $VARS; do   # each variant's source hash (sidecar of the build), so a log names what it compared
  echo "variant $v: $(libof $v) source $(cat $(libof $v).srchash 2>/dev/null || echo unknown) md5 $(md5sum < $(libof $v) | cut -c1-12)"
  BMPC_LIBRARY=$(libof $v) timeout -k 10 150 python tools/variant_check.py $out/vc_$v.npz $QB || exit 1   # same B N NB as the timed runs
done
OUT=$out VARS="$VARS" python - <<'PY'
import os
import numpy as np
o = os.environ["OUT"]; vs = os.environ["VARS"].split()
a = np.load(f"{o}/vc_{vs[0]}.npz")
for tag in vs[1:]:
    b = np.load(f"{o}/vc_{tag}.npz")
    print(tag, "vs", vs[0], "status agree %.4f  #0 %d -> %d  iters mean %.2f -> %.2f  max |dJ|/|J| %.2e  max |du0| %.2e" % (
        np.mean(a["status"] == b["status"]), (a["status"] == 0).sum(), (b["status"] == 0).sum(), a["iters"].mean(),
        b["iters"].mean(), np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"]))),
        np.max(np.abs(a["upred"][:, 0] - b["upred"][:, 0]))), flush=True)
PY
: > $out/time.log
for rep in 1 2; do
  for v in $VARS; do
    echo "== $v" >> $out/time.log
    BMPC_LIBRARY=$(libof $v) timeout -k 10 150 python tools/quick_bench.py $QB 2>&1 | grep "^step [123]" | cut -c1-110 >> $out/time.log || exit 1
  done
done
python - $out/time.log <<'PY'
import re, sys, collections
cur = None; d = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    m = re.match(r"== (\S+)", ln)
    if m: cur = m.group(1); continue
    m = re.search(r"ipm ([\d.]+) ms", ln)
    if m: d[cur].append(float(m.group(1)))
for k, v in d.items():
    print(f"TIME {k}: k_ipm mean {sum(v)/len(v):.2f} ms  min {min(v):.2f}  (n={len(v)})")
PY
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    BMPC_LIBRARY=$(libof $v) timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $out/p_${v}_$c -o run --output-format csv \
      -- python3 $R/tools/quick_bench.py $QB > $out/p_${v}_$c.log 2>&1 || exit 1
  done
done
python3 - $out "$VARS" <<'PY'
import csv, glob, sys, collections
out, vs = sys.argv[1], sys.argv[2].split()
for v in vs:
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = collections.defaultdict(float)
        for f in glob.glob(f"{out}/p_{v}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_ipm" in r["Kernel_Name"] or "k_solve" in r["Kernel_Name"]:
                    per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        vals = sorted(per.items(), key=lambda t: int(t[0]))[1:]   # drop the cold first solve
        res[c] = sum(x for _, x in vals) / max(len(vals), 1)
    gb = (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024 / 1e9
    print(f"PMC {v}: FETCH {res['FETCH_SIZE']*1024/1e9:.1f} GB  WRITE {res['WRITE_SIZE']*1024/1e9:.1f} GB  2F+W {gb:.1f} GB per warm k_ipm launch")
PY
find $out -name "*.csv" -delete
find $out -type f -size +2M -delete   # keep what comes back under the 64 MiB merge limit
