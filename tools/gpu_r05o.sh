#!/bin/bash
# round 5: where one ego's time goes on the small-batch kernel: the -DBMPC_PROFILE phase split
# at one ego (N=20 NB=1, N=8 NB=2) and the SQ instruction mix of the product kernel at one ego
set -o pipefail
o=$PWD/gpurun_out/${1:-r05o}
mkdir -p $o
R=$PWD
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 150 python tools/phase_profile.py 1 20 1 > $o/pp1_n20.log 2>&1 || exit $?
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 150 python tools/phase_profile.py 1 8 2 > $o/pp1_n8.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace -d $o/sq1 -o run --output-format csv -- python3 $R/tools/quick_bench.py 1 20 1 > $o/sq1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_FLAT --kernel-trace -d $o/sq2 -o run --output-format csv -- python3 $R/tools/quick_bench.py 1 20 1 > $o/sq2.log 2>&1 || exit $?
python3 - $o <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for d in ("sq1", "sq2"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_solve_blk" in r["Kernel_Name"]:
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, v in per.items():
        vals = [x for _, x in sorted(v.items(), key=lambda t: int(t[0]))][1:]
        print(f"{c:24s} per warm dispatch {sum(vals)/max(len(vals),1):.4e}  (n={len(vals)})")
PY
find $o -name "*.csv" -delete
cat $o/pp1_n20.log $o/pp1_n8.log
