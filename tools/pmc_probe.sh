#!/bin/bash
# rocprofv3 counter passes over one quick_bench launch sequence (4096 highway egos): one pass per
# argument (a space-separated counter list, within the per-block limits of
# MI355X_MICROARCH.md), each its own run; per-dispatch averages of the IPM kernel, cold first
# solve dropped.  usage: bash tools/pmc_probe.sh TAG "C1 C2" "C3" ...
# (QB_ARGS: quick_bench arguments "B N NB", default 4096; KF: kernel-name regex, default k_ipm|k_solve)
tag=$1; shift
R=$PWD
out=$R/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for cs in "$@"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $cs --kernel-trace -d $out/p$i -o run --output-format csv \
    -- python3 $R/tools/quick_bench.py ${QB_ARGS:-4096} > $out/p$i.log 2>&1
  echo "pass $i ($cs): rc $?" >> $out/summary.txt
done
python3 - $out "${KF:-k_ipm|k_solve}" >> $out/summary.txt <<'PY'
import csv, glob, re, sys, collections
out, kf = sys.argv[1], re.compile(sys.argv[2])
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kf.search(r["Kernel_Name"]):
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
for c, d in sorted(per.items()):
    vals = [v for _, v in sorted(d.items())][1:] or list(d.values())
    print(f"{c:40s} {sum(vals) / len(vals):.4e}  (dispatches {len(vals)})")
PY
find $out -name "*.csv" -delete
cat $out/summary.txt
