#!/bin/bash
# Calibration pass on the GPU box (tools/mb_calib.hip, built in-tree beforehand):
# FETCH_SIZE / WRITE_SIZE of known byte counts at 8 and 16 B per lane, the scratch cost of a
# call's callee-saved registers, and the price of a kernel boundary (stream launches, hipGraph).
# usage: bash tools/gpu_calib.sh TAG
set -o pipefail
tag=${1:-calib}
out=$PWD/gpurun_out/${tag}
mkdir -p $out
MB=$PWD/tools/mb_calib
timeout -k 10 60 $MB launch 4096 > $out/launch.log 2>&1 || exit $?
timeout -k 10 60 $MB launch 256 >> $out/launch.log 2>&1 || exit $?
cat $out/launch.log
cd /tmp && export TMPDIR=/tmp
for m in fetch8 fetch16 write8 write16 scratch; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --kernel-trace -d $out/$m-$c -o run --output-format csv -- $MB $m \
      > $out/$m-$c.log 2>&1 || exit $?
  done
done
python3 - $out <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(out + "/*-*_SIZE")):
    m, c = d.rsplit("/", 1)[1].split("-")
    vals = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        vals += list(per.values())
    res.setdefault(m, {})[c + "_kB_per_dispatch"] = vals
print(json.dumps(res, indent=1))
json.dump(res, open(out + "/calib.json", "w"), indent=1)
PY
find $out -name "*.csv" -delete
