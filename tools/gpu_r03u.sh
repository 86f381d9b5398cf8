#!/bin/bash
# round-3 pass u: band-QP single-problem latency, kernel trace and PC sampling of k_bandqp
set -o pipefail
mkdir -p gpurun_out/r03u
out=$PWD/gpurun_out/r03u
timeout -k 10 120 python tools/qp_lat.py 30 > $out/lat.log 2>&1 || exit $?
cat $out/lat.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- \
   python3 $GRAFT_REPO_ROOT/tools/qp_lat.py 30 > $out/kt.log 2>&1) || exit $?
f=$(find $out/kt -name "*kernel_stats.csv" | head -1); cat "$f"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
   --pc-sampling-unit time --pc-sampling-interval 50 -d $out/pcs -o run --output-format csv -- \
   python3 $GRAFT_REPO_ROOT/tools/qp_lat.py 60 > $out/pcs.log 2>&1) || exit $?
python3 - $out/pcs <<'PY'
import csv, glob, sys, collections
fs = glob.glob(sys.argv[1] + "/**/*pc_sampling*.csv", recursive=True)
print(fs)
c = collections.Counter(); tot = 0
for f in fs:
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "") or ""
        if "bandqp" not in k: continue
        ins = r.get("Instruction", "") or r.get("Inst", "")
        c[(r.get("Instruction_Comment", "")[:60], ins[:50])] += 1; tot += 1
print("samples", tot)
for (cm, ins), n in c.most_common(60): print(f"{n:7d} {100*n/max(tot,1):5.1f}%  {ins:50s} {cm}")
PY
find $out -name "*.csv" -size +2M -delete
echo done
