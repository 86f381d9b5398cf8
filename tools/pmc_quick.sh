#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / TCC hit-miss of the IPM kernel in separate rocprofv3 passes (dev helper)
# usage: tools/pmc_quick.sh TAG [bench args]
tag=${1:-q}; shift
out=$PWD/gpurun_out/pmc_${tag}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  d=$out/$(echo $c | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d $d -o run --output-format csv -- python3 $B --no-cpu-baseline --steps 2 --warmup 1 "$@" > $d.log 2>&1 || exit $?
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_ipm" not in k and "k_qp" not in k: continue
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, d in agg.items():
    print(c, "per dispatch avg", sum(d.values()) / len(d), "dispatches", len(d))
PY
find $out -name "*.csv" -delete
