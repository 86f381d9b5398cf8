#!/bin/bash
# GPU box: k_ipm time and HBM bytes at reduced occupancy (BMPC_IPM_LDS_BYTES reserves LDS per ego,
# so fewer egos are resident per CU: a smaller working set per L2).  Seeded 4096-ego headline batch
# (tools/quick_bench.py), libbmpc.so or LIB=<path>.  usage: bash tools/occ_sweep.sh TAG "0 13600 20400 40960"
set -o pipefail
tag=${1:-occ}
R=$PWD
out=$R/gpurun_out/$tag
mkdir -p $out
LIB=${LIB:-$R/belief-planning_amd/libbmpc.so}
: > $out/time.log
for b in ${2:-0 13600 20400 40960}; do
  echo "== lds $b" >> $out/time.log
  BMPC_LIBRARY=$LIB BMPC_IPM_LDS_BYTES=$b timeout -k 10 150 python tools/quick_bench.py 4096 2>&1 | grep "^step [123]" | cut -c1-110 >> $out/time.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
for b in ${2:-0 13600 20400 40960}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    BMPC_LIBRARY=$LIB BMPC_IPM_LDS_BYTES=$b timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $out/p_${b}_$c -o run --output-format csv \
      -- python3 $R/tools/quick_bench.py 4096 > $out/p_${b}_$c.log 2>&1 || exit 1
  done
done
python3 - $out "${2:-0 13600 20400 40960}" <<'PY'
import csv, glob, re, sys, collections
out, bs = sys.argv[1], sys.argv[2].split()
t = collections.defaultdict(list); cur = None
for ln in open(f"{out}/time.log"):
    m = re.match(r"== lds (\d+)", ln)
    if m: cur = m.group(1); continue
    m = re.search(r"ipm ([\d.]+) ms", ln)
    if m: t[cur].append(float(m.group(1)))
for b in bs:
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = collections.defaultdict(float)
        for f in glob.glob(f"{out}/p_{b}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_ipm" in r["Kernel_Name"]:
                    per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        vals = sorted(per.items(), key=lambda kv: int(kv[0]))[1:]
        res[c] = sum(x for _, x in vals) / max(len(vals), 1)
    gb = (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024 / 1e9
    v = t[b]
    print(f"LDS {b:>6s} B/ego: k_ipm {sum(v)/max(len(v),1):.2f} ms (steps 1-3)  2F+W {gb:.1f} GB per warm launch")
PY
find $out -name "*.csv" -delete
